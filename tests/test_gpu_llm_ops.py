"""GPU numerics of the LM kernels against plain PyTorch fp32 references.

fused linear+CE (cross_entropy.hip), RoPE + SwiGLU (rope_swiglu.hip).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V", [50257, 1000, 32000])
def test_fused_linear_ce_matches_fp32_reference(dtype, V):
    from hyperion.ops.cross_entropy import fused_linear_cross_entropy

    torch.manual_seed(0)
    N, E, pad = 300, 256, V - 1
    x = (torch.randn(N, E, device="cuda") * 0.5).to(dtype).requires_grad_(True)
    w = (torch.randn(V, E, device="cuda") * 0.05).to(dtype).requires_grad_(True)
    b = (torch.randn(V, device="cuda") * 0.1).to(dtype).requires_grad_(True)
    t = torch.randint(0, V, (N,), device="cuda")
    t[::7] = pad  # ignored rows
    loss = fused_linear_cross_entropy(x, w, b, t, ignore_index=pad)
    loss.backward()
    xr, wr, br = (a.detach().float().requires_grad_(True) for a in (x, w, b))
    ref = F.cross_entropy(F.linear(xr, wr, br), t, ignore_index=pad)
    ref.backward()
    tol = dict(rtol=1e-4, atol=1e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(loss.float(), ref, **tol)
    gt = dict(rtol=1e-3, atol=1e-5) if dtype == torch.float32 else dict(rtol=5e-2, atol=3e-3)
    torch.testing.assert_close(x.grad.float(), xr.grad, **gt)
    torch.testing.assert_close(w.grad.float(), wr.grad, **gt)
    torch.testing.assert_close(b.grad.float(), br.grad, **gt)


@pytest.mark.parametrize("chunk", [8192, 1000])
def test_fused_linear_ce_no_logits_path(chunk, monkeypatch):
    """The bf16 path that never stores the [N, V] logits (LSE epilogue pass + per-chunk softmax-
    gradient epilogue passes) runs, matches the fp32 reference, and its peak extra memory stays
    well below the logits' size (LM-256 shape: 4064 tokens x 50257 classes, E = 256)."""
    import hyperion.ops.cross_entropy as hce
    from hyperion.ops import _native

    monkeypatch.setattr(hce, "CE_CHUNK", chunk)
    monkeypatch.setattr(hce, "CE_MATERIALIZE_BYTES", 0)
    torch.manual_seed(0)
    N, E, V, pad = 4064, 256, 50257, 50256
    x = (torch.randn(N, E, device="cuda") * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(V, E, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    b = (torch.randn(V, device="cuda") * 0.1).requires_grad_(True)
    t = torch.randint(0, V - 1, (N,), device="cuda")
    t[::9] = pad
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    _native.reset_counters()
    loss = hce.fused_linear_cross_entropy(x, w, b, t, ignore_index=pad)
    loss.backward()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    assert _native.counters().get("linear_ce_fused") == 1
    assert peak < 0.6 * N * V * 2, peak  # the bf16 logits alone would be 408 MB
    xr, wr, br = (a.detach().float().requires_grad_(True) for a in (x, w, b))
    ref = F.cross_entropy(F.linear(xr, wr, br), t, ignore_index=pad)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, rtol=2e-2, atol=2e-2)
    for got, want in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (got.float() - want).norm() <= 3e-2 * want.norm() + 1e-6


@pytest.mark.parametrize("N,E,with_bias", [(4064, 256, True), (2032, 768, True), (300, 128, False)])
def test_fused_linear_ce_materialized_path(N, E, with_bias):
    """The default bf16 schedule: bf16 logits (rows padded to 8 classes), register-resident
    in-place CE with the bias added in the kernel, dX on the tiled split-K GEMM + odd-tail update,
    dW on hipBLASLt — against the fp32 reference (LM-256 / GPT-2 head shapes, V = 50257)."""
    import hyperion.ops.cross_entropy as hce
    from hyperion.ops import _native

    torch.manual_seed(0)
    V, pad = 50257, 50256
    x = (torch.randn(N, E, device="cuda") * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(V, E, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    b = (torch.randn(V, device="cuda") * 0.1).bfloat16().requires_grad_(True) if with_bias else None
    t = torch.randint(0, V, (N,), device="cuda")
    t[::9] = pad
    _native.reset_counters()
    loss = hce.fused_linear_cross_entropy(x, w, b, t, ignore_index=pad)
    (loss * 0.5).backward()  # a non-unit incoming gradient
    assert _native.counters().get("linear_ce_materialized") == 1
    leaves = (x, w) + ((b,) if with_bias else ())
    refs = [a.detach().float().requires_grad_(True) for a in leaves]
    ref = F.cross_entropy(F.linear(refs[0], refs[1], refs[2] if with_bias else None), t, ignore_index=pad)
    (ref * 0.5).backward()
    torch.testing.assert_close(loss.float(), ref, rtol=2e-2, atol=2e-2)
    for got, want in zip(leaves, refs):
        assert (got.grad.float() - want.grad).norm() <= 3e-2 * want.grad.norm() + 1e-6


@pytest.mark.parametrize("ld_pad", [0, 7, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_ce_kernel_bias_and_row_layouts(ld_pad, dtype):
    """ce_fwd_bwd with an fp32 bias on aligned rows (register-resident kernel) and on odd row
    strides (two-pass kernel) equals the fp32 softmax-CE of z + b and its gradient."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(3)
    N, V = 67, 5003
    buf = (torch.randn(N, V + ld_pad, device="cuda") * 3).to(dtype)
    z = buf[:, :V]
    bias = torch.randn(V, device="cuda")
    t = torch.randint(0, V, (N,), device="cuda")
    t[5] = -100
    scale = torch.full((1,), 1.0 / N, device="cuda")
    zr = (z.float() + bias).requires_grad_(True)
    ref = F.cross_entropy(zr, t, ignore_index=-100, reduction="sum") / N
    ref.backward()
    lse_ref = torch.logsumexp(zr.detach(), 1)
    loss_rows, lse = C.ce_fwd_bwd(z, t, scale, 1.0, -100, True, bias)
    torch.testing.assert_close(loss_rows.sum() / N, ref, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(lse, lse_ref, rtol=1e-4, atol=1e-4)
    tol = dict(rtol=1e-3, atol=1e-6) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-4)
    torch.testing.assert_close(z.float(), zr.grad, **tol)


def test_fused_linear_ce_chunked_equals_unchunked():
    from hyperion.ops.cross_entropy import fused_linear_cross_entropy

    torch.manual_seed(1)
    x = torch.randn(257, 64, device="cuda", requires_grad=True)
    w = torch.randn(999, 64, device="cuda", requires_grad=True)
    t = torch.randint(0, 999, (257,), device="cuda")
    l1 = fused_linear_cross_entropy(x, w, None, t)
    g1 = torch.autograd.grad(l1, (x, w))
    l2 = fused_linear_cross_entropy(x, w, None, t, max_logits_bytes=999 * 4 * 50)  # 50-row chunks
    g2 = torch.autograd.grad(l2, (x, w))
    torch.testing.assert_close(l1, l2)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("D", [64, 128])
def test_rope_matches_reference(dtype, D):
    from hyperion.ops.rope import apply_rope, rope_reference

    torch.manual_seed(0)
    B, S, H = 2, 77, 4
    q = torch.randn(B, S, H, D, device="cuda", dtype=dtype, requires_grad=True)
    k = torch.randn(B, S, H, D, device="cuda", dtype=dtype, requires_grad=True)
    qo, ko = apply_rope(q, k, None, 10000.0)
    qr, kr = (a.detach().float().requires_grad_(True) for a in (q, k))
    qro, kro = rope_reference(qr, kr, None, 10000.0)
    tol = dict(rtol=1e-4, atol=5e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(qo.float(), qro, **tol)
    torch.testing.assert_close(ko.float(), kro, **tol)
    gq, gk = torch.randn_like(qo), torch.randn_like(ko)
    (qo * gq).sum().add((ko * gk).sum()).backward()
    (qro * gq.float()).sum().add((kro * gk.float()).sum()).backward()
    torch.testing.assert_close(q.grad.float(), qr.grad, **tol)
    torch.testing.assert_close(k.grad.float(), kr.grad, **tol)


def test_rope_positions_argument():
    from hyperion.ops.rope import apply_rope, rope_reference

    q = torch.randn(1, 8, 2, 64, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, 8, 2, 64, device="cuda", dtype=torch.bfloat16)
    pos = torch.tensor([[5, 6, 7, 8, 100, 200, 300, 4000]], device="cuda")
    qo, ko = apply_rope(q, k, pos)
    qr, kr = rope_reference(q.float(), k.float(), pos)
    torch.testing.assert_close(qo.float(), qr, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_swiglu_matches_reference(dtype):
    from hyperion.ops.swiglu import swiglu

    torch.manual_seed(0)
    g = torch.randn(33, 344, device="cuda", dtype=dtype, requires_grad=True)
    u = torch.randn(33, 344, device="cuda", dtype=dtype, requires_grad=True)
    h = swiglu(g, u)
    gr, ur = (a.detach().float().requires_grad_(True) for a in (g, u))
    hr = F.silu(gr) * ur
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(h.float(), hr, **tol)
    dh = torch.randn_like(h)
    h.backward(dh)
    hr.backward(dh.float())
    torch.testing.assert_close(g.grad.float(), gr.grad, **tol)
    torch.testing.assert_close(u.grad.float(), ur.grad, **tol)


def test_llama_tiny_native_matches_torch_path(monkeypatch):
    from hyperion.models.llama import LlamaConfig, LlamaForCausalLM

    torch.manual_seed(0)
    cfg = LlamaConfig.tiny(hidden_size=256, num_attention_heads=2, intermediate_size=512)
    m = LlamaForCausalLM(cfg).cuda().to(torch.bfloat16)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), device="cuda")
    mask = torch.ones_like(ids)
    mask[1, 50:] = 0
    labels = ids.masked_fill(mask == 0, -100)
    out = m(ids, attention_mask=mask, labels=labels)
    out.loss.backward()
    g_native = [p.grad.float().clone() for p in m.parameters()]
    m.zero_grad(set_to_none=True)
    monkeypatch.setenv("HYPERION_KERNELS", "torch")
    ref = m(ids, attention_mask=mask, labels=labels)
    ref.loss.backward()
    torch.testing.assert_close(out.loss.float(), ref.loss.float(), rtol=2e-2, atol=2e-2)
    for a, p in zip(g_native, m.parameters()):
        b = p.grad.float()
        assert (a - b).norm() <= 0.1 * b.norm() + 1e-3


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_linear_act_matches_reference(act):
    from hyperion.ops.linear_act import linear_act

    torch.manual_seed(0)
    x = torch.randn(4, 33, 64, device="cuda", requires_grad=True)
    w = torch.randn(128, 64, device="cuda", requires_grad=True)
    b = torch.randn(128, device="cuda", requires_grad=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = linear_act(x, w, b, act)
    y.float().square().sum().backward()
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    yr = F.relu(yr) if act == "relu" else F.gelu(yr)
    yr.square().sum().backward()
    assert (y.float() - yr).norm() <= 2e-2 * yr.norm()
    for a, r in ((x, xr), (w, wr), (b, br)):
        assert (a.grad.float() - r.grad).norm() <= 0.03 * r.grad.norm()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_native_dropout_mask_stats_and_backward(dt):
    """Counter-based dropout: keep rate 1-p, kept values scaled by 1/(1-p), the backward applies
    exactly the forward's mask (regenerated, never stored), and consecutive calls draw new masks."""
    from hyperion.ops import _native
    from hyperion.ops.dropout import dropout

    torch.manual_seed(0)
    p = 0.1
    x = (torch.rand(4096, 1000, device="cuda") + 0.5).to(dt).requires_grad_(True)
    _native.reset_counters()
    y = dropout(x, p, True)
    assert _native.counters().get("dropout") == 1
    keep = y != 0
    assert abs(keep.float().mean().item() - (1 - p)) < 2e-3
    torch.testing.assert_close(y[keep].float(), (x[keep].float() / (1 - p)).to(dt).float())
    g = torch.randn_like(x)
    y.backward(g)
    torch.testing.assert_close(x.grad, (g.float() * keep.float() / (1 - p)).to(dt))
    y2 = dropout(x.detach(), p, True)
    assert ((y2 != 0) != keep).float().mean().item() > 0.1  # a fresh mask


def test_native_dropout_fresh_mask_per_graph_replay():
    """Under hipGraph capture the seed/offset are read from torch's generator state at replay time:
    every replay draws a new mask (the old host-seed scheme replayed the captured one)."""
    from hyperion.ops.dropout import dropout

    x = torch.ones(1 << 16, device="cuda", dtype=torch.bfloat16)
    out = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out.copy_(dropout(x, 0.5, True))
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_(dropout(x, 0.5, True))
    g.replay()
    torch.cuda.synchronize()
    m1 = out.clone()
    g.replay()
    torch.cuda.synchronize()
    assert not torch.equal(m1, out)
    assert abs((out != 0).float().mean().item() - 0.5) < 0.02


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_post_norm_layer_residual_grad_rides_the_gemm(monkeypatch, p):
    """Post-norm encoder layer: each norm's residual gradient is added in the epilogue of the data
    gradient GEMM of the layer input's other consumer (QKV, linear1) instead of an autograd add —
    same gradients as the unlinked layer (ops/linear.py arm_link / take_link_grad)."""
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.ops import _native
    from hyperion.ops import conv as conv_mod

    torch.manual_seed(0)
    layer = TransformerEncoderLayer(256, 4, 1024, dropout=p, activation="gelu").cuda().bfloat16()
    x0 = torch.randn(4, 64, 256, device="cuda").bfloat16()
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(conv_mod, "FUSE_SHORTCUT_GRAD", fuse)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        _native.reset_counters()
        torch.manual_seed(1)
        _native.rng_state(x.device)  # (same dropout stream for both runs)
        y = layer(x, causal=True)
        (y.float() * torch.linspace(-1, 1, 256, device="cuda")).sum().backward()
        torch.cuda.synchronize()
        res.append((y.detach().clone(), x.grad.clone(), {n: q.grad.clone() for n, q in layer.named_parameters()},
                    dict(_native.counters())))
    assert res[1][3].get("residual_grad_fused") == 2 and not res[0][3].get("residual_grad_fused")
    if p == 0.0:
        assert torch.equal(res[0][0], res[1][0])
        torch.testing.assert_close(res[1][1].float(), res[0][1].float(), rtol=2e-2, atol=2e-2)
        for n in res[0][2]:  # (the attention backward's atomics make both runs differ at bf16 level)
            a, b = res[1][2][n].float(), res[0][2][n].float()
            assert float((a - b).norm() / (b.norm() + 1e-12)) < 1e-2, n


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_post_norm_layer_bias_grads_from_norm_backward(monkeypatch, p):
    """out_proj's and linear2's bias gradients come from the LayerNorm backward kernel's column sums
    of the branch gradient (BiasGradLink, layernorm.hip BSUM) — equal to summing dy separately."""
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.ops import _native
    from hyperion.ops import layernorm as ln_mod

    torch.manual_seed(0)
    layer = TransformerEncoderLayer(256, 4, 1024, dropout=p, activation="gelu").cuda().bfloat16()
    x0 = torch.randn(4, 64, 256, device="cuda").bfloat16()
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(ln_mod, "FUSE_BIAS_GRAD", fuse)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        _native.reset_counters()
        torch.cuda.manual_seed(123)  # the same dropout masks in both runs
        y = layer(x, causal=True)
        (y.float() * torch.linspace(-1, 1, 256, device="cuda")).sum().backward()
        torch.cuda.synchronize()
        res.append(({n: q.grad.clone() for n, q in layer.named_parameters()}, dict(_native.counters())))
    assert res[1][1].get("bias_grad_from_norm") == 2 and not res[0][1].get("bias_grad_from_norm")
    for n in ("self_attn.out_proj.bias", "linear2.bias"):
        a, b = res[1][0][n].float(), res[0][0][n].float()
        assert float((a - b).norm() / (b.norm() + 1e-12)) < 2e-2, n


@pytest.mark.parametrize("ckpt", [False, True])
def test_vit_bias_grads_from_norm_backward(monkeypatch, ckpt):
    """ViT pre-norm blocks: out_proj (via ln_2) and fc2 (via the next block's ln_1 / the final ln)
    bias gradients from the LayerNorm backward's column sums — same gradients as summing dy."""
    from hyperion.models.vit import VisionTransformer
    from hyperion.ops import _native
    from hyperion.ops import layernorm as ln_mod

    torch.manual_seed(0)
    m = VisionTransformer(64, 16, 3, 4, 256, 512, num_classes=10, use_checkpoint=ckpt).cuda().bfloat16()
    x0 = torch.randn(4, 3, 64, 64, device="cuda").bfloat16()
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(ln_mod, "FUSE_BIAS_GRAD", fuse)
        m.zero_grad(set_to_none=True)
        _native.reset_counters()
        m(x0).float().square().mean().backward()
        torch.cuda.synchronize()
        res.append(({n: q.grad.clone() for n, q in m.named_parameters() if q.grad is not None},
                    dict(_native.counters())))
    if not ckpt:
        assert res[1][1].get("bias_grad_from_norm") == 6, res[1][1]
    assert not res[0][1].get("bias_grad_from_norm")
    for n in res[0][0]:
        a, b = res[1][0][n].float(), res[0][0][n].float()
        assert float((a - b).norm() / (b.norm() + 1e-12)) < 2e-2, n


def test_ln_bwd_branch_sums_in_bias_dtype():
    """fp32 LayerNorm weights (cast_for_compute keeps norms fp32) with a bf16 producing linear: the
    branch-gradient sums come out of the same combine in bf16 (``bsum_dtype``) — no cast kernel —
    and equal the column sums of the returned gradient; dγ / dβ stay fp32."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(0)
    rows, d = 1000, 768
    x = torch.randn(rows, d, device="cuda").bfloat16()
    w = torch.randn(d, device="cuda") * 0.5 + 1.0
    b = torch.randn(d, device="cuda") * 0.1
    y, _, mean, rstd = C.ln_fwd(x, None, w, b, 1e-5, False)
    dy = torch.randn(rows, d, device="cuda").bfloat16()
    ref = C.ln_bwd(dy, x, w, mean, rstd, None, True, True, False, 0.0, None, True)
    out = C.ln_bwd(dy, x, w, mean, rstd, None, True, True, False, 0.0, None, True, _native.DTYPE_CODE[torch.bfloat16])
    dx, dw, db, _, dbs = out
    assert dbs.dtype == torch.bfloat16 and dw.dtype == torch.float32 and db.dtype == torch.float32
    assert ref[4].dtype == torch.float32  # default: the weight dtype, packed after dγ | dβ
    torch.testing.assert_close(dx, ref[0], rtol=0, atol=0)
    torch.testing.assert_close(dw, ref[1], rtol=0, atol=0)
    torch.testing.assert_close(db, ref[2], rtol=0, atol=0)
    torch.testing.assert_close(dbs.float(), ref[4].bfloat16().float(), rtol=0, atol=0)
    torch.testing.assert_close(dbs.float(), dx.float().sum(0), rtol=2e-2, atol=2e-2)


def test_vit_compute_copies_bias_grads_without_cast(monkeypatch):
    """ViT with bf16 compute copies and fp32 norms (the bench's cast_for_compute): the fused bias
    gradients arrive in the bias dtype and match the unfused column sums."""
    from hyperion.models.vit import VisionTransformer
    from hyperion.ops import _native
    from hyperion.ops import layernorm as ln_mod
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = VisionTransformer(64, 16, 3, 4, 256, 512, num_classes=10).cuda()
    cast_for_compute(m, torch.bfloat16)
    assert m.encoder.ln.weight.dtype == torch.float32 and m.heads.head.weight.dtype == torch.bfloat16
    x0 = torch.randn(4, 3, 64, 64, device="cuda").bfloat16()
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(ln_mod, "FUSE_BIAS_GRAD", fuse)
        m.zero_grad(set_to_none=True)
        _native.reset_counters()
        m(x0).float().square().mean().backward()
        torch.cuda.synchronize()
        res.append(({n: q.grad.clone() for n, q in m.named_parameters() if q.grad is not None},
                    dict(_native.counters())))
    assert res[1][1].get("bias_grad_from_norm") == 6, res[1][1]
    params = dict(m.named_parameters())
    for n in res[0][0]:
        a, b = res[1][0][n], res[0][0][n]
        assert a.dtype == params[n].dtype, n
        assert float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)) < 2e-2, n


@pytest.mark.parametrize("N,E", [(2032, 768), (4064, 256)])
def test_lm_head_all_native_gemms(N, E):
    """HYPERION_GEMM=native: the V = 50257 head runs every GEMM on the tiled kernel — logits as
    classes [0, 50256) + one launch for the last class and the row padding (weight rows past V read
    as zeros), dX reducing over 50257 classes (ragged last slice staged per lane), dW over the padded
    class rows — and matches the fp32 reference; the padding columns of the logits are exact zeros."""
    import hyperion.ops.cross_entropy as hce
    from hyperion.ops import _native, gemm

    torch.manual_seed(1)
    V, pad = 50257, 50256
    x = (torch.randn(N, E, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(V, E, device="cuda") * 0.05).bfloat16()
    gemm.set_mode("native")
    try:
        zb = torch.full((N, 50264), float("nan"), device="cuda", dtype=torch.bfloat16)
        assert gemm.lm_head_logits(x, w, zb)
        ref = x.float() @ w.float().t()
        torch.testing.assert_close(zb[:, :V].float(), ref, rtol=2e-2, atol=2e-2)
        assert torch.equal(zb[:, V:], torch.zeros_like(zb[:, V:]))
        dz = (torch.randn(N, V, device="cuda") * 0.01).bfloat16()
        zb[:, :V] = dz
        dx = gemm.lm_head_dx(zb, w)
        torch.testing.assert_close(dx.float(), dz.float() @ w.float(), rtol=2e-2, atol=2e-2)
        xr = x.detach().float().requires_grad_(True)
        wr = w.detach().float().requires_grad_(True)
        xg, wg = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        t = torch.randint(0, V, (N,), device="cuda")
        t[::9] = pad
        _native.reset_counters()
        loss = hce.fused_linear_cross_entropy(xg, wg, None, t, ignore_index=pad)
        loss.backward()
        cnt = _native.counters()
        assert cnt.get("gemm_lm_head") == 1 and cnt.get("gemm_lm_head_dx") == 1 and cnt.get("gemm_tn", 0) >= 1, cnt
        refl = F.cross_entropy(F.linear(xr, wr), t, ignore_index=pad)
        refl.backward()
        torch.testing.assert_close(loss.float(), refl, rtol=2e-2, atol=2e-2)
        for got, want in ((xg.grad, xr.grad), (wg.grad, wr.grad)):
            assert (got.float() - want).norm() <= 3e-2 * want.norm() + 1e-6
    finally:
        gemm.set_mode("auto")


def test_gemm_ragged_k_and_b_rows():
    """K % 8 != 0 with one transposed operand (the other's row padding finite) and n_out > rows of
    B (zero columns past them), on the fast tiles and the SAFE tile."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(2)
    M, N, K = 1000, 768, 1001
    buf = torch.randn(M, 1008, device="cuda").bfloat16()
    buf[:, K:] = 7.0  # finite padding: multiplied by the zero rows of B past K
    a = buf[:, :K]
    b = torch.randn(K, N, device="cuda").bfloat16()
    ref = a.float() @ b.float()
    for tile in (0, 2, 3, 8, 11):
        for sp in (1, 3):
            c = C.gemm(a, b, b_tr=True, out_dtype=torch.float32, tile=tile, splits=sp)
            torch.testing.assert_close(c, ref, rtol=1e-4, atol=2e-2, msg=f"tile {tile} splits {sp}")
    w = torch.randn(5, 256, device="cuda").bfloat16()
    xa = torch.randn(300, 256, device="cuda").bfloat16()
    out = torch.full((300, 8), float("nan"), device="cuda", dtype=torch.bfloat16)
    C.gemm(xa, w, out=out, n_out=8)
    torch.testing.assert_close(out[:, :5].float(), xa.float() @ w.float().t(), rtol=2e-2, atol=2e-2)
    assert torch.equal(out[:, 5:], torch.zeros_like(out[:, 5:]))


def test_vit_selective_recompute_matches_and_saves_memory():
    """use_checkpoint="selective": LayerNorm and GELU outputs are rebuilt in backward from recipes
    (ops/recompute.py) instead of being saved by the next GEMM — same gradients as the plain step
    (the LN recompute is the same kernel; GELU comes from the fused GELU pass instead of the GEMM
    epilogue: rounding-level differences), recipes really used, and lower peak memory."""
    from hyperion.models.vit import VisionTransformer
    from hyperion.ops import recompute

    torch.manual_seed(0)
    m = VisionTransformer(64, 16, 4, 4, 256, 1024, num_classes=10).cuda().bfloat16()
    x0 = torch.randn(32, 3, 64, 64, device="cuda").bfloat16()
    res = {}
    for mode in (False, "selective", True):
        m.use_checkpoint = mode
        m.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        recompute.STATS.update(packed=0, recomputed=0)
        m(x0).float().square().mean().backward()
        torch.cuda.synchronize()
        res[mode] = ({n: q.grad.float().clone() for n, q in m.named_parameters()},
                     torch.cuda.max_memory_allocated() - base, dict(recompute.STATS))
    g0, peak0, _ = res[False]
    gs, peaks, st = res["selective"]
    # ln_1, ln_2, gelu outputs (one save each) and the attention output (saved by attention AND out_proj)
    assert st["packed"] >= 4 * 5 and st["recomputed"] == 4 * 4, st
    assert peaks < peak0, (peaks, peak0)
    for n in g0:
        assert float((gs[n] - g0[n]).norm() / (g0[n].norm() + 1e-12)) < 2e-2, n
