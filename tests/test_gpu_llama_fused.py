"""The fused Llama LoRA layer (ops/llama_fused.py) and its kernels against torch references.

Reference workload: ``train_llama_fsdp(lora=True)`` (``02_development/distributed_utils.py:463-476``):
frozen bf16 Llama + PEFT LoRA r16 on q/k/v/o.  Checks: the weight-streaming epilogues (LoRA up +
RoPE, SwiGLU fwd/bwd, LoRA data gradient), the rank-r kernels, and the whole fused decoder layer vs
the module path and vs an fp32 torch model.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from hyperion.ops import _native

    return _native.native()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_lora_rank_r_kernels_match_fp32():
    torch.manual_seed(0)
    C = _C()
    M, K, N, r, P = 100, 512, 256, 16, 3
    bf = torch.bfloat16
    x = torch.randn(M, K, device="cuda", dtype=bf)
    A = [torch.randn(r, K, device="cuda", dtype=bf) * 0.1 for _ in range(P)]
    t = torch.zeros(M, P * r, device="cuda")
    C.lora_down(x, A, t)
    ref = torch.cat([x.float() @ a.float().t() for a in A], 1)
    assert _rel(t, ref) < 1e-2
    dy = torch.randn(M, P * N, device="cuda", dtype=bf)
    B = [torch.randn(N, r, device="cuda", dtype=bf) * 0.1 for _ in range(P)]
    dB = [torch.empty_like(b) for b in B]
    du = torch.zeros(M, P * r, device="cuda")
    C.lora_bwd_t(dy, N, B, dB, t, du, 1.5)
    for p in range(P):
        dyp = dy[:, p * N:(p + 1) * N].float()
        assert _rel(du[:, p * r:(p + 1) * r], 1.5 * dyp @ B[p].float()) < 1e-2
        assert _rel(dB[p], 1.5 * dyp.t() @ t[:, p * r:(p + 1) * r]) < 2e-2
    dA = [torch.empty_like(a) for a in A]
    C.lora_bwd_a(x, dA, du)
    for p in range(P):
        assert _rel(dA[p], du[:, p * r:(p + 1) * r].t() @ x.float()) < 2e-2


@pytest.mark.parametrize("splits", [2, 4])
def test_lora_rank_r_split_stacks_match_fp32(splits):
    """t / du as split-partial stacks [S, M, W] (what the fused layer uses): lora_down and lora_bwd_t
    write one slice per split, every consumer sums them."""
    torch.manual_seed(1)
    C = _C()
    M, K, N, r, P = 128, 1024, 512, 16, 3
    bf = torch.bfloat16
    x = torch.randn(M, K, device="cuda", dtype=bf)
    A = [torch.randn(r, K, device="cuda", dtype=bf) * 0.1 for _ in range(P)]
    t = torch.full((splits, M, 4 * r), float("nan"), device="cuda")[:, :, :P * r]
    C.lora_down(x, A, t)
    ref_t = torch.cat([x.float() @ a.float().t() for a in A], 1)
    assert _rel(t.sum(0), ref_t) < 1e-2
    dy = torch.randn(M, P * N, device="cuda", dtype=bf)
    B = [torch.randn(N, r, device="cuda", dtype=bf) * 0.1 for _ in range(P)]
    dB = [torch.empty_like(b) for b in B]
    du = torch.full((splits, M, 4 * r), float("nan"), device="cuda")[:, :, :P * r]
    C.lora_bwd_t(dy, N, B, dB, t, du, 1.5)
    tsum = t.sum(0)
    for p in range(P):
        dyp = dy[:, p * N:(p + 1) * N].float()
        assert _rel(du.sum(0)[:, p * r:(p + 1) * r], 1.5 * dyp @ B[p].float()) < 1e-2
        assert _rel(dB[p], 1.5 * dyp.t() @ tsum[:, p * r:(p + 1) * r]) < 2e-2
    dA = [torch.empty_like(a) for a in A]
    C.lora_bwd_a(x, dA, du)
    for p in range(P):
        assert _rel(dA[p], du.sum(0)[:, p * r:(p + 1) * r].t() @ x.float()) < 2e-2


def test_lora_dropout_mask_rate_and_regeneration():
    """keep rate 1 - p; the same rng record regenerates the same mask in every kernel."""
    from hyperion.ops import _native

    torch.manual_seed(0)
    C = _C()
    M, K, r = 128, 4096, 16
    x = torch.ones(M, K, device="cuda", dtype=torch.bfloat16)
    A = [torch.ones(r, K, device="cuda", dtype=torch.bfloat16)]
    rs = _native.rng_state(x.device)
    t1 = torch.zeros(M, r, device="cuda")
    C.lora_down(x, A, t1, rs, 0.05)
    rate = (t1[:, 0] / K).mean().item()
    assert abs(rate - 0.95) < 0.005, rate
    t2 = torch.zeros(M, r, device="cuda")
    C.lora_down(x, A, t2, rs, 0.05)
    assert torch.equal(t1, t2)
    # dA with du = 1 counts kept elements per column: Σ_k over columns equals Σ of t (same mask)
    du = torch.ones(M, r, device="cuda")
    dA = [torch.empty(r, K, device="cuda", dtype=torch.float32).bfloat16()]
    C.lora_bwd_a(x, dA, du, rs, 0.05)
    assert abs(dA[0][0].float().sum().item() - t1[:, 0].sum().item()) <= 0.01 * t1[:, 0].sum().item()


def _slabs(x, w, nn=False):
    return _C().ws_gemm_part(x, w, nn=nn)


def test_ws_epilogue_lora_up_rope():
    from hyperion.ops.rope import rope_reference

    torch.manual_seed(1)
    C = _C()
    Bz, S, nh, hd = 2, 48, 2, 128
    H, M, r = nh * hd, Bz * S, 16
    x = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(3 * H, H, device="cuda", dtype=torch.bfloat16) * 0.05
    t = torch.randn(M, 3 * r, device="cuda")
    Bs = [torch.randn(H, r, device="cuda", dtype=torch.bfloat16) * 0.1 for _ in range(3)]
    part, nS, MFt = _slabs(x, w)
    out = torch.empty(M, 3 * H, device="cuda", dtype=torch.bfloat16)
    C.ws_epilogue(part, nS, MFt, M, 3 * H, 1, out, t=t, lw=Bs, segw=H, lscale=2.0, rope_segs=2, seq=S)
    y = x.float() @ w.float().t()
    for p in range(3):
        y[:, p * H:(p + 1) * H] += 2.0 * t[:, p * r:(p + 1) * r] @ Bs[p].float().t()
    y = y.bfloat16().view(Bz, S, 3, nh, hd)
    qr, kr = rope_reference(y[:, :, 0], y[:, :, 1], None)
    o5 = out.view(Bz, S, 3, nh, hd)
    assert _rel(o5[:, :, 0], qr) < 1e-2 and _rel(o5[:, :, 1], kr) < 1e-2 and _rel(o5[:, :, 2], y[:, :, 2]) < 1e-2


def test_ws_epilogue_swiglu_fwd_bwd():
    torch.manual_seed(2)
    C = _C()
    M, H, I = 100, 256, 512
    x = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    wgu = torch.randn(2 * I, H, device="cuda", dtype=torch.bfloat16) * 0.05
    part, nS, MFt = _slabs(x, wgu)
    gu = torch.empty(M, 2 * I, device="cuda", dtype=torch.bfloat16)
    h = torch.empty(M, I, device="cuda", dtype=torch.bfloat16)
    C.ws_epilogue(part, nS, MFt, M, 2 * I, 2, gu, out2=h)
    z = (x.float() @ wgu.float().t()).bfloat16().float()
    assert _rel(gu, z) < 1e-2
    assert _rel(h, F.silu(z[:, :I]) * z[:, I:]) < 1e-2
    dd = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
    wd = torch.randn(H, I, device="cuda", dtype=torch.bfloat16) * 0.05
    part, nS, MFt = _slabs(dd, wd, nn=True)
    dgu = torch.empty(M, 2 * I, device="cuda", dtype=torch.bfloat16)
    C.ws_epilogue(part, nS, MFt, M, I, 3, dgu, aux=gu)
    dh = (dd.float() @ wd.float()).bfloat16().float()
    g, u = gu[:, :I].float().requires_grad_(True), gu[:, I:].float().requires_grad_(True)
    (F.silu(g) * u).backward(dh)
    assert _rel(dgu[:, :I], g.grad) < 2e-2 and _rel(dgu[:, I:], u.grad) < 2e-2


def test_ws_epilogue_lora_dgrad_no_dropout():
    torch.manual_seed(3)
    C = _C()
    M, H, r = 64, 256, 16
    dy = torch.randn(M, 3 * H, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(3 * H, H, device="cuda", dtype=torch.bfloat16) * 0.05
    du = torch.randn(M, 3 * r, device="cuda")
    As = [torch.randn(r, H, device="cuda", dtype=torch.bfloat16) * 0.1 for _ in range(3)]
    part, nS, MFt = _slabs(dy, w, nn=True)
    out = torch.empty(M, H, device="cuda", dtype=torch.bfloat16)
    C.ws_epilogue(part, nS, MFt, M, H, 4, out, t=du, lw=As)
    ref = dy.float() @ w.float() + sum(du[:, p * r:(p + 1) * r] @ As[p].float() for p in range(3))
    assert _rel(out, ref) < 1e-2


def _tiny_lora_llama(p_drop=0.0, seed=0):
    from hyperion.models.llama import LlamaConfig, LlamaForCausalLM
    from hyperion.models.lora import apply_lora
    from hyperion.ops.llama_fused import fuse_llama_weights

    torch.manual_seed(seed)
    cfg = LlamaConfig.tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=2, intermediate_size=512)
    m = LlamaForCausalLM(cfg).cuda().to(torch.bfloat16)
    apply_lora(m, r=16, alpha=32, dropout=p_drop)
    with torch.no_grad():  # non-zero B so every adapter gradient is exercised
        for n, p in m.named_parameters():
            if ".lora_B." in n:
                p.normal_(0, 0.02)
    fuse_llama_weights(m)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), device="cuda")
    mask = torch.ones_like(ids)
    mask[1, 50:] = 0
    return m, ids, mask


def _run(m, ids, mask):
    m.zero_grad(set_to_none=True)
    out = m(ids, attention_mask=mask, labels=ids)
    out.loss.backward()
    return out.loss.detach().float(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.requires_grad}


def test_fused_llama_layer_matches_module_path(monkeypatch):
    import hyperion.models.llama as L
    from hyperion.ops import _native

    m, ids, mask = _tiny_lora_llama()
    _native.reset_counters()
    loss_f, g_f = _run(m, ids, mask)
    assert _native.counters().get("llama_fused_layer", 0) >= 2, _native.counters()
    monkeypatch.setattr(L, "FUSED", False)
    loss_m, g_m = _run(m, ids, mask)
    assert abs(loss_f.item() - loss_m.item()) <= 2e-2 * abs(loss_m.item())
    for n in g_m:
        assert _rel(g_f[n], g_m[n]) < 0.06, n


def test_fused_llama_lora_grads_vs_fp32_torch(monkeypatch):
    """bf16 fused LoRA gradients against the same model evaluated in fp32 by plain torch ops."""
    import copy

    m, ids, mask = _tiny_lora_llama()
    loss_f, g_f = _run(m, ids, mask)
    ref = copy.deepcopy(m).float()
    monkeypatch.setenv("HYPERION_KERNELS", "torch")
    loss_r, g_r = _run(ref, ids, mask)
    assert abs(loss_f.item() - loss_r.item()) <= 2e-2 * abs(loss_r.item())
    for n in g_r:
        assert _rel(g_f[n], g_r[n]) < 0.06, n


def test_fused_llama_lora_dropout_active_and_replayable():
    m, ids, mask = _tiny_lora_llama(p_drop=0.05)
    m.train()
    torch.manual_seed(123)
    l1, g1 = _run(m, ids, mask)
    torch.manual_seed(123)
    l2, g2 = _run(m, ids, mask)
    assert abs(l1.item() - l2.item()) < 1e-3
    for n in g1:
        assert _rel(g1[n], g2[n]) < 1e-3, n  # same rng state -> same masks (fp32 atomics order only)
    m.eval()  # eval: no dropout
    l3, g3 = _run(m, ids, mask)
    assert any(_rel(g1[n], g3[n]) > 1e-3 for n in g1 if ".lora_A." in n)
