"""Round-4 native paths vs plain fp32 PyTorch references.

* the ResNet RGB stem (7x7/s2/p3, C=3) on the native conv kernels: ``stem.hip`` space-to-depth
  (exact copy of the torch reference rewrite), then conv_fwd / conv_wgrad as a stride-1 R=4 conv
  with a 16-element pixel stride — forward, BN statistics and weight gradient against fp32
  ``F.conv2d`` + BN + ReLU (reference stem: torchvision ResNet conv1 on MIOpen,
  ``Phase 1/baseline_performance.ipynb:203-205``).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 3, 224, 224), (3, 3, 33, 31), (1, 4, 17, 18), (2, 1, 64, 64)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_stem_s2d_kernel_is_the_reference_rewrite(shape, dtype):
    from hyperion.ops import _native
    from hyperion.ops.conv import stem_s2d_reference

    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    got = _native.native().stem_s2d(x)
    ref = stem_s2d_reference(x)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, ref)  # a pure gather: bit-exact


@pytest.mark.parametrize("C", [1, 3, 4])
@pytest.mark.parametrize("cl", [False, True])
def test_stem_weight_transforms_one_launch_match_reference(C, cl):
    """stem_weight4 / stem_weight4_grad (one launch each) == the torch index-gather forms, bitwise,
    for either weight layout; dW comes back in the weight's own layout."""
    from hyperion.ops import _native
    from hyperion.ops.conv import stem_weight, stem_weight_grad

    torch.manual_seed(0)
    w = torch.randn(64, C, 7, 7, device="cuda").bfloat16()
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    N = _native.native()
    w4 = N.stem_weight4(w)
    ref = stem_weight(w).contiguous(memory_format=torch.channels_last)
    assert w4.is_contiguous(memory_format=torch.channels_last) and torch.equal(w4, ref)
    dw4 = torch.randn(64, 64, 4, 1, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dw = N.stem_weight4_grad(dw4, C, cl)
    assert torch.equal(dw, stem_weight_grad(dw4, C))
    assert dw.is_contiguous(memory_format=torch.channels_last) == cl or C == 1


@pytest.mark.parametrize("N,H", [(4, 64), (2, 224)])
def test_stem_conv_bn_relu_native_matches_fp32(N, H):
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act

    torch.manual_seed(0)
    _native.reset_counters()
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda()
    bn = BatchNormAct2d(64, act=True).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    conv_l = conv.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(N, 3, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = conv_bn_act(conv_l, bn, x)
    g = torch.randn_like(out)
    out.backward(g)
    cnt = _native.counters()
    assert cnt.get("stem_s2d") == 1 and cnt.get("conv_bn_act") == 1 and "conv_bn_act_fallback" not in cnt, cnt
    assert cnt.get("wgrad") == 1 and "wgrad_vendor" not in cnt, cnt
    wr = conv_l.weight.detach().float().cpu().requires_grad_(True)
    y = F.conv2d(x.float().cpu(), wr, stride=2, padding=3)
    y = F.relu(F.batch_norm(y, None, None, bn.weight.detach().cpu(), bn.bias.detach().cpu(), True, 0.1, bn.eps))
    y.backward(g.float().cpu())
    torch.testing.assert_close(out.float().cpu(), y.detach(), rtol=3e-2, atol=3e-2)
    dw = conv_l.weight.grad.float().cpu()
    assert dw.shape == wr.grad.shape
    torch.testing.assert_close(dw, wr.grad, rtol=3e-2, atol=3e-2 * wr.grad.abs().max().item())


# ---- stride-2 data gradient as 4 output-phase sub-convolutions in one launch (conv_igemm.hip sd2)
S2_SHAPES = [  # N, C (dX channels), H (dX), K (dY channels), R, pad
    (2, 128, 16, 128, 3, 1),
    (3, 64, 14, 64, 3, 1),
    (1, 64, 8, 256, 3, 1),
    (2, 256, 28, 256, 3, 1),
    (2, 64, 12, 128, 5, 2),
]


@pytest.mark.parametrize("shape", S2_SHAPES)
@pytest.mark.parametrize("with_add", [False, True])
def test_strided_dgrad_phases_match_fp32(shape, with_add):
    from hyperion.ops import _native

    N, C, H, K, R, p = shape
    torch.manual_seed(0)
    P = (H + 2 * p - R) // 2 + 1
    assert 2 * P == H
    dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") / (K * R * R) ** 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    add = (torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
           if with_add else None)
    dx = _native.native().conv_dgrad(dy, w, p, p, addend=add, stride=2, H=H, W=H)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().cpu(), dy.float().cpu(), stride=2, padding=p)
    if with_add:
        ref = ref + add.float().cpu()
    assert dx.shape == ref.shape and dx.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(dx.float().cpu(), ref, rtol=2e-2, atol=2e-2)


def _strided_chain(fuse_bn_backward):
    from hyperion.ops import _native
    from hyperion.ops import conv as convmod
    from hyperion.ops.batchnorm import BatchNormAct2d

    torch.manual_seed(0)
    _native.reset_counters()
    prev, convmod.FUSE_BN_BACKWARD = convmod.FUSE_BN_BACKWARD, fuse_bn_backward
    try:
        c1 = torch.nn.Conv2d(64, 128, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        b1 = BatchNormAct2d(128, act=True).cuda()
        c2 = torch.nn.Conv2d(128, 128, 3, stride=2, padding=1, bias=False).cuda().to(torch.bfloat16).to(
            memory_format=torch.channels_last)
        b2 = BatchNormAct2d(128, act=True).cuda()
        x = torch.randn(2, 64, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        out = convmod.conv_bn_act(c2, b2, convmod.conv_bn_act(c1, b1, x))
        out.backward(torch.randn(out.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(5)).to(
            out.dtype).contiguous(memory_format=torch.channels_last))
    finally:
        convmod.FUSE_BN_BACKWARD = prev
    return x.grad.float(), c1.weight.grad.float(), c2.weight.grad.float(), _native.counters()


def test_strided_conv_bn_act_backward_native_bn_epilogue():
    """A stride-2 3x3 conv -> BN -> ReLU fed by another fused layer: its data gradient runs the
    native phase kernel WITH the producer's BN-backward epilogue (no vendor dgrad), and equals the
    same chain with the epilogue off (separate BN-backward reduce) — the same bf16 math."""
    gx, g1, g2, cnt = _strided_chain(True)
    assert cnt.get("dgrad_strided") == 1 and cnt.get("dgrad_bn_fused") == 1 and "dgrad_vendor" not in cnt, cnt
    rx, r1, r2, cnt0 = _strided_chain(False)
    assert cnt0.get("dgrad_strided") == 1 and "dgrad_bn_fused" not in cnt0, cnt0
    for a, b in ((gx, rx), (g1, r1), (g2, r2)):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2 * b.abs().max().item())


def test_strided_conv_bn_act_leaf_input_matches_fp32():
    """The strided layer alone (leaf input: plain phase dgrad) against fp32 PyTorch."""
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act
    import torch.nn.functional as F

    torch.manual_seed(0)
    _native.reset_counters()
    c2 = torch.nn.Conv2d(128, 256, 3, stride=2, padding=1, bias=False).cuda().to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    b2 = BatchNormAct2d(256, act=False).cuda()
    x = torch.randn(2, 128, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    out = conv_bn_act(c2, b2, x)
    g = torch.randn_like(out)
    out.backward(g)
    assert _native.counters().get("dgrad_strided") == 1, _native.counters()
    xr = x.detach().float().cpu().requires_grad_(True)
    wr = c2.weight.detach().float().cpu().requires_grad_(True)
    y = F.batch_norm(F.conv2d(xr, wr, stride=2, padding=1), None, None, b2.weight.detach().cpu(),
                     b2.bias.detach().cpu(), True)
    y.backward(g.float().cpu())
    torch.testing.assert_close(x.grad.float().cpu(), xr.grad, rtol=3e-2, atol=3e-2 * xr.grad.abs().max().item())


# ---- dropout fused into LayerNorm (residual branch) and into the FFN's GEMM epilogue / act backward
def _same_state(fn_fused, fn_unfused):
    """Run both with the default generator in the same state (the fused op draws one rng record,
    the unfused composition draws the identical record for its dropout)."""
    g = torch.cuda.default_generators[torch.cuda.current_device()]
    st = g.get_state()
    a = fn_fused()
    g.set_state(st)
    b = fn_unfused()
    return a, b


@pytest.mark.parametrize("d", [256, 512, 768])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_layernorm_dropout_fused_matches_unfused(d, dt):
    from hyperion.ops import _native
    from hyperion.ops.dropout import dropout
    from hyperion.ops.layernorm import layer_norm

    torch.manual_seed(0)
    p = 0.1
    x0 = torch.randn(4, 37, d, device="cuda").to(dt)
    r0 = torch.randn(4, 37, d, device="cuda").to(dt)
    w = (torch.rand(d, device="cuda") + 0.5).requires_grad_(True)
    b = (torch.randn(d, device="cuda") * 0.1).requires_grad_(True)
    g = torch.randn(4, 37, d, device="cuda").to(dt)

    def run(fused):
        x = x0.clone().requires_grad_(True)
        r = r0.clone().requires_grad_(True)
        w.grad = b.grad = None
        if fused:
            y = layer_norm(x, w, b, 1e-5, residual=r, dropout_p=p)
        else:
            y = layer_norm(dropout(x, p), w, b, 1e-5, residual=r)
        y.backward(g)
        return y.float(), x.grad.float(), r.grad.float(), w.grad.clone(), b.grad.clone()

    _native.reset_counters()
    fu, un = _same_state(lambda: run(True), lambda: run(False))
    assert _native.counters().get("ln_dropout") == 1 and _native.counters().get("dropout") == 1
    for a, c in zip(fu, un):
        torch.testing.assert_close(a, c, rtol=1e-2, atol=1e-2)
    frac = (fu[1] == 0).float().mean().item()  # dropped elements get no gradient
    assert 0.05 < frac < 0.15, frac


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("force", ["native", "vendor"])
def test_linear_act_dropout_fused_matches_unfused(act, force):
    from hyperion.ops import gemm
    from hyperion.ops.dropout import dropout
    from hyperion.ops.linear_act import linear_act

    torch.manual_seed(0)
    p = 0.1
    gemm.set_mode(force)
    try:
        x0 = torch.randn(512, 256, device="cuda").bfloat16()
        w = (torch.randn(1024, 256, device="cuda") * 0.05).requires_grad_(True)
        b = (torch.randn(1024, device="cuda") * 0.1).requires_grad_(True)
        g = torch.randn(512, 1024, device="cuda").bfloat16()

        def run(fused):
            x = x0.clone().requires_grad_(True)
            w.grad = b.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                if fused:
                    h = linear_act(x, w, b, act, dropout_p=p)
                else:
                    h = dropout(linear_act(x, w, b, act), p)
            h.backward(g)
            return h.float(), x.grad.float(), w.grad.clone(), b.grad.clone()

        fu, un = _same_state(lambda: run(True), lambda: run(False))
    finally:
        gemm.set_mode("auto")
    for a, c in zip(fu, un):
        torch.testing.assert_close(a, c, rtol=2e-2, atol=2e-2 * max(1.0, c.abs().max().item()))


def test_fused_dropout_masks_regenerate_under_graph_replay():
    """A captured post-norm encoder layer (LN + FFN dropouts fused) draws a fresh mask on every
    replay, and no standalone dropout kernel is left in the layer."""
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.ops import _native

    torch.manual_seed(0)
    layer = TransformerEncoderLayer(256, 4, 1024, dropout=0.1).cuda().train()
    x = torch.randn(8, 64, 256, device="cuda")
    _native.reset_counters()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        layer(x)
    cnt = _native.counters()
    assert cnt.get("ln_dropout") == 2 and "dropout" not in cnt, cnt
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.autocast("cuda", dtype=torch.bfloat16):
        layer(x)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr), torch.autocast("cuda", dtype=torch.bfloat16):
        out = layer(x)
    gr.replay()
    a = out.clone()
    gr.replay()
    b = out.clone()
    assert not torch.equal(a, b)  # fresh masks per replay
    layer.eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        e1, e2 = layer(x), layer(x)
    assert torch.equal(e1, e2)  # eval: no dropout


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gelu_dropout_one_pass_matches_fp32(p, dt):
    """dropout.hip mode 2 (the vendor-GEMM FFN path: exact-erf GELU + dropout in one pass) against
    fp32 GELU times the same call's scaled keep mask; odd element count exercises the scalar tail."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(0)
    z = (torch.randn(1001, 77, device="cuda") * 3).to(dt)
    st = _native.rng_state(z.device) if p > 0 else None
    h = C.dropout(z, p, st, act=2)
    keep = C.dropout(torch.ones_like(z), p, st, mask=True).float() if p > 0 else 1.0
    ref = torch.nn.functional.gelu(z.float()) * keep
    torch.testing.assert_close(h.float(), ref, rtol=1e-2, atol=1e-2)
    if p > 0:  # (GELU itself is exactly 0 below about -5.5 in fp32: count the mask, not h)
        frac = float((keep == 0).float().mean())
        assert abs(frac - p) < 0.02


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_fused_mse_loss_matches_fp32(dt):
    """ops.losses.MSELoss (one native pass: mean + gradient 2(x - t)/n) vs nn.MSELoss in fp32."""
    from hyperion.ops import _native
    from hyperion.ops.losses import MSELoss

    torch.manual_seed(0)
    x = torch.randn(32, 1000, device="cuda").to(dt).requires_grad_(True)
    t = torch.rand(32, 1000, device="cuda")
    _native.reset_counters()
    loss = MSELoss()(x, t)
    (loss * 3.0).backward()
    assert _native.counters().get("mse_fused") == 1
    xr = x.detach().float().requires_grad_(True)
    ref = torch.nn.functional.mse_loss(xr, t)
    (ref * 3.0).backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-6)


def test_weight_hook_sees_reduced_wgrad():
    """A tensor hook on a conv weight receives the final weight gradient: the split-K wgrad reduce
    is not deferred past it (ops/conv.py _can_defer), so the hooked value equals .grad."""
    from hyperion.models.resnet import resnet18
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    seen = {}
    w = m.layer1[0].conv1.weight
    w.register_hook(lambda g: seen.__setitem__("g", g.detach().clone()))
    x = torch.randn(8, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    m(x).float().square().mean().backward()
    torch.cuda.synchronize()
    assert "g" in seen and torch.equal(seen["g"], w.grad)


@pytest.mark.parametrize("shape", [(8, 64, 28, 256, 1, 1, 0), (8, 128, 14, 128, 3, 1, 1), (4, 256, 14, 512, 1, 2, 0),
                                   (3, 64, 9, 64, 3, 1, 1)])
@pytest.mark.parametrize("tile", [(64, 64), (128, 64), (128, 128)])
def test_conv_fwd_direct_store_epilogue_bitwise(shape, tile):
    """The DIRECT forward epilogue (accumulator lane pairs stored straight to global, stages + 16)
    writes the same output and BN-statistics sums as the LDS-transposed store epilogue, bit for bit
    (same rounding, same summation order), including partial edge tiles."""
    from hyperion.ops import _native

    C = _native.native()
    N, Cin, H, K, R, s, p = shape
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, Cin, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for stages in (2, 18):
        sums = torch.zeros(_native.STAT_SLOTS * 2 * K, device="cuda", dtype=torch.float64)
        y = C.conv_fwd(x, w, s, s, p, p, True, tile[0], tile[1], 1, sums=sums, stages=stages)[0]
        outs.append((y.clone(), sums.clone()))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-12, atol=1e-9)  # f64 atomics: order may vary
    ref = torch.nn.functional.conv2d(x.float(), w.float(), stride=s, padding=p)
    torch.testing.assert_close(outs[1][0].float(), ref, rtol=2e-2, atol=2e-2)
