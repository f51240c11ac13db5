"""Horizontally fused data + weight gradient launch (csrc/kernels/conv_dual.hip).

* op level: ``conv_dgrad_wgrad`` returns the SAME dX / dz (bitwise) as ``conv_dgrad`` and the same
  dW as ``conv_wgrad`` with the 64 x 64 plan, for every geometry the ResNets use (1x1 dense short /
  long reductions, 3x3 stride 1, 3x3 stride 2 by output phase, 1x1 stride 2 on the output grid),
  with and without the BN-backward epilogue (LEAN mode 1, full mode 2 + addend), both grid orders;
  and both are close to the fp32 torch gradients of the same conv;
* the deferred split-K reduce chain: a fused launch that defers its dW reduce, the next fused
  launch running it as extra workgroups, then a flush — dW equals the standalone reduce;
* model level: a ResNet-50 backward with the fused launches (``wgrad_dual`` dispatches) gives the
  gradients of the separate launches to within the BN statistics' run-to-run atomics noise.

Reference: MIOpen bwd-data / bwd-weights as separate kernels (SURVEY §2.4 conv row).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, C, H, K, R, stride, pad): the conv's input [N, C, H, H], filter [K, C, R, R]
SHAPES = [
    (8, 64, 56, 256, 1, 1, 0),    # layer1 expand 1x1: long dense reduction (M = 25088)
    (4, 256, 14, 64, 1, 1, 0),    # short dense
    (4, 64, 28, 64, 3, 1, 1),     # 3x3 stride 1
    (4, 128, 28, 128, 3, 2, 1),   # 3x3 stride 2 (the phase-split data gradient)
    (4, 256, 28, 512, 1, 2, 0),   # 1x1 stride 2 downsample (data gradient on the output grid)
]


def _t(shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).bfloat16().contiguous(memory_format=torch.channels_last)


def _case(shape, seed=0):
    N, C, H, K, R, s, p = shape
    g = torch.Generator(device="cuda").manual_seed(seed)
    P = (H + 2 * p - R) // s + 1
    x = (torch.randn(N, C, H, H, device="cuda", generator=g)).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda", generator=g) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = (torch.randn(N, K, P, P, device="cuda", generator=g)).bfloat16().contiguous(memory_format=torch.channels_last)
    return x, w, dy


def _dgrad_kw(shape, x):
    N, C, H, K, R, s, p = shape
    if s == 2 and R > 1:
        return dict(ph=p, pw=p, stride=2, H=H, W=H)
    if s == 2:
        return dict(ph=0, pw=0)  # 1x1 strided: the stride-1 GEMM on the output grid
    return dict(ph=p, pw=p)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("order", [0, 1])
def test_dual_matches_separate_launches(shape, order):
    from hyperion.ops import _native

    C_ = _native.native()
    N, C, H, K, R, s, p = shape
    x, w, dy = _case(shape)
    kw = _dgrad_kw(shape, x)
    ph, pw = kw.pop("ph"), kw.pop("pw")
    dx_ref = C_.conv_dgrad(dy, w, ph, pw, **kw)
    dw_ref = C_.conv_wgrad(dy, x, R, R, s, s, p, p, 64, 64)
    dx, dw = C_.conv_dgrad_wgrad(dy, w, ph, pw, wg_x=x, wg_R=R, wg_S=R, wg_sh=s, wg_sw=s, wg_ph=p, wg_pw=p,
                                 order=order, **kw)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    assert torch.equal(dw, dw_ref)
    # and against fp32 torch (guards against both paths being wrong the same way)
    dw32 = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), stride=s, padding=p)
    rel = ((dw.float() - dw32).norm() / dw32.norm()).item()
    assert rel < 2e-2, rel
    if not (s == 2 and R == 1):
        dx32 = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), stride=s, padding=p)
        rel = ((dx.float() - dx32).norm() / dx32.norm()).item()
        assert rel < 2e-2, rel


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("shape", [SHAPES[0], SHAPES[2], SHAPES[3]])
def test_dual_bn_backward_epilogue(shape, mode):
    """The data gradient with the producing BN layer's backward epilogue (dz = dX·mask, Σdz, Σdz·x):
    dz bitwise equal to the separate launch, the sums equal to the fp64 atomics' noise."""
    from hyperion.ops import _native

    C_ = _native.native()
    N, C, H, K, R, s, p = shape
    x, w, dy = _case(shape, seed=1)
    kw = _dgrad_kw(shape, x)
    ph, pw = kw.pop("ph"), kw.pop("pw")
    g = torch.Generator(device="cuda").manual_seed(5)
    yc = torch.randn(x.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    bw = torch.rand(C, device="cuda", generator=g) + 0.5
    bb = torch.randn(C, device="cuda", generator=g) * 0.1
    mean = torch.randn(C, device="cuda", generator=g) * 0.1
    invstd = torch.rand(C, device="cuda", generator=g) + 0.5
    xout = torch.relu(yc.float() * (bw * invstd).view(1, -1, 1, 1) + (bb - mean * bw * invstd).view(1, -1, 1, 1))
    xout = xout.bfloat16().contiguous(memory_format=torch.channels_last)
    add = _t(x.shape) if mode == 2 else None
    slots = _native.STAT_SLOTS

    def bnkw(sums):
        return dict(addend=add, bn_x=yc, bn_y=xout if mode == 2 else None, bn_w=bw, bn_b=bb, bn_mean=mean,
                    bn_invstd=invstd, bn_mode=mode, bn_sums=sums)

    s1 = torch.zeros(slots * 2 * C, device="cuda", dtype=torch.float64)
    s2 = torch.zeros_like(s1)
    dz_ref = C_.conv_dgrad(dy, w, ph, pw, **bnkw(s1), **kw)
    dw_ref = C_.conv_wgrad(dy, x, R, R, s, s, p, p, 64, 64)
    dz, dw = C_.conv_dgrad_wgrad(dy, w, ph, pw, wg_x=x, wg_R=R, wg_S=R, wg_sh=s, wg_sw=s, wg_ph=p, wg_pw=p,
                                 **bnkw(s2), **kw)
    torch.cuda.synchronize()
    assert torch.equal(dz, dz_ref)
    assert torch.equal(dw, dw_ref)
    a, b = s1.view(slots, 2, C).sum(0), s2.view(slots, 2, C).sum(0)
    torch.testing.assert_close(b, a, rtol=1e-9, atol=1e-9 * a.abs().max().item())


def test_dual_deferred_reduce_chain():
    """dW's split-K reduce deferred by one fused launch runs in the next one's extra workgroups."""
    from hyperion.ops import _native

    C_ = _native.native()
    sh1, sh2 = SHAPES[0], SHAPES[2]
    x1, w1, dy1 = _case(sh1, seed=2)
    x2, w2, dy2 = _case(sh2, seed=3)
    ref1 = C_.conv_wgrad(dy1, x1, 1, 1, 1, 1, 0, 0, 64, 64)
    ref2 = C_.conv_wgrad(dy2, x2, 3, 3, 1, 1, 1, 1, 64, 64)
    assert not C_.conv_wgrad_flush()
    _, dw1 = C_.conv_dgrad_wgrad(dy1, w1, 0, 0, wg_x=x1, wg_R=1, wg_S=1, wg_sh=1, wg_sw=1, wg_ph=0, wg_pw=0,
                                 wg_defer=True)
    _, dw2 = C_.conv_dgrad_wgrad(dy2, w2, 1, 1, wg_x=x2, wg_R=3, wg_S=3, wg_sh=1, wg_sw=1, wg_ph=1, wg_pw=1,
                                 wg_defer=True)  # runs dw1's reduce, defers its own
    assert C_.conv_wgrad_flush()  # dw2's reduce
    torch.cuda.synchronize()
    assert torch.equal(dw1, ref1)
    assert torch.equal(dw2, ref2)


def test_dual_resnet50_backward_matches_separate():
    """A whole ResNet-50 backward with the fused launches vs separate ones: same gradients to the
    BN statistics atomics' run-to-run noise; the fused launch served nearly every layer."""
    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import resnet50
    from hyperion.ops import _native
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = resnet50(num_classes=16).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 16, device="cuda").bfloat16()

    def run(dual):
        prev, prevf = hconv._DUAL, hconv.WGRAD_FUSE
        hconv._DUAL, hconv.WGRAD_FUSE = dual, "dgrad"
        try:
            for q in m.parameters():
                q.grad = None
            _native.reset_counters()
            m(x0).backward(gy)
            torch.cuda.synchronize()
            return [q.grad.float().clone() for q in m.parameters()], _native.counters()
        finally:
            hconv._DUAL, hconv.WGRAD_FUSE = prev, prevf

    (ref, c0), (ref2, _), (got, c1) = run("0"), run("0"), run("1")
    assert c0.get("wgrad_dual", 0) == 0
    assert c1.get("wgrad_dual", 0) >= 50, c1  # every conv but the stem (52 of 53)
    for u, u2, v in zip(ref, ref2, got):
        noise = (u2 - u).norm().item()
        assert (v - u).norm().item() <= 4 * noise + 1e-2 * u.norm().item() + 1e-6


# ---- BN dx pass + the weight gradient of the conv above it (csrc/kernels/bn_wgrad.hip) ----------
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("tile", [(64, 64), (128, 64), (64, 128)])
def test_bn_dx_wgrad_matches_separate(shape, tile):
    """bn_bwd_dx_wgrad == bn_bwd_dx + conv_wgrad (same tile / split plan), bitwise, for every conv
    geometry of the ResNets; the BN layer is a different tensor (the layer below)."""
    from hyperion.ops import _native

    C_ = _native.native()
    N, C, H, K, R, s, p = shape
    if C % tile[1] != 0:
        pytest.skip("bn must divide C")
    x, w, dy = _case(shape, seed=4)
    g = torch.Generator(device="cuda").manual_seed(9)
    Cb = 128
    dz = torch.randn(N, Cb, 20, 20, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    yc = torch.randn(N, Cb, 20, 20, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    bw = torch.rand(Cb, device="cuda", generator=g) + 0.5
    mean = torch.randn(Cb, device="cuda", generator=g) * 0.1
    invstd = torch.rand(Cb, device="cuda", generator=g) + 0.5
    sums = torch.randn(_native.STAT_SLOTS * 2 * Cb, device="cuda", generator=g, dtype=torch.float64)
    dx_ref, dbw_ref, dbb_ref = C_.bn_bwd_dx(dz, yc, bw, mean, invstd, True, sums)
    dw_ref = C_.conv_wgrad(dy, x, R, R, s, s, p, p, tile[0], tile[1])
    out = torch.full(w.shape, 7.0, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dx, dbw, dbb, dw = C_.bn_bwd_dx_wgrad(dz, yc, bw, mean, invstd, True, sums, wg_dy=dy, wg_x=x, wg_R=R, wg_S=R,
                                          wg_sh=s, wg_sw=s, wg_ph=p, wg_pw=p, wg_bm=tile[0], wg_bn=tile[1], wg_out=out)
    torch.cuda.synchronize()
    assert dw.data_ptr() == out.data_ptr()  # written in place
    assert torch.equal(dx, dx_ref) and torch.equal(dbw, dbw_ref) and torch.equal(dbb, dbb_ref)
    assert torch.equal(dw, dw_ref)


def test_bn_dx_wgrad_deferred_chain():
    """The fused launch runs an earlier deferred split-K reduce and defers its own; a flush ends it."""
    from hyperion.ops import _native

    C_ = _native.native()
    x1, w1, dy1 = _case(SHAPES[0], seed=6)
    x2, w2, dy2 = _case(SHAPES[2], seed=7)
    ref1 = C_.conv_wgrad(dy1, x1, 1, 1, 1, 1, 0, 0, 64, 64)
    ref2 = C_.conv_wgrad(dy2, x2, 3, 3, 1, 1, 1, 1, 64, 64)
    dz = _t((4, 64, 28, 28))
    yc = _t((4, 64, 28, 28))
    ones, zeros = torch.ones(64, device="cuda"), torch.zeros(64, device="cuda")
    sums = torch.zeros(_native.STAT_SLOTS * 2 * 64, device="cuda", dtype=torch.float64)
    assert not C_.conv_wgrad_flush()
    dw1 = C_.conv_wgrad(dy1, x1, 1, 1, 1, 1, 0, 0, 64, 64, defer=True)
    _, _, _, dw2 = C_.bn_bwd_dx_wgrad(dz, yc, ones, zeros, ones, True, sums, wg_dy=dy2, wg_x=x2, wg_R=3, wg_S=3,
                                      wg_sh=1, wg_sw=1, wg_ph=1, wg_pw=1, wg_defer=True)
    assert C_.conv_wgrad_flush()
    torch.cuda.synchronize()
    assert torch.equal(dw1, ref1)
    assert torch.equal(dw2, ref2)


@pytest.mark.parametrize("fuse", ["bn", "dgrad"])
def test_wgrad_fusion_resnet50_backward_matches_separate(fuse):
    """A ResNet-50 backward with parked weight gradients riding on the next BN dx pass ("bn") or on
    their own data gradient ("dgrad") vs separate launches: same gradients to the BN atomics' noise,
    and the fused launches served most layers."""
    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import resnet50
    from hyperion.ops import _native
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = resnet50(num_classes=16).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 16, device="cuda").bfloat16()

    def run(mode):
        prev = hconv.WGRAD_FUSE
        hconv.WGRAD_FUSE = mode
        try:
            for q in m.parameters():
                q.grad = None
            _native.reset_counters()
            m(x0).backward(gy)
            torch.cuda.synchronize()
            assert hconv._parked["req"] is None and not hconv._defer_state["pending"]
            return [q.grad.float().clone() for q in m.parameters()], _native.counters()
        finally:
            hconv.WGRAD_FUSE = prev

    (ref, c0), (ref2, _), (got, c1) = run("0"), run("0"), run(fuse)
    assert c0.get("wgrad_bn_fused", 0) == 0 and c0.get("wgrad_dual", 0) == 0
    key = "wgrad_bn_fused" if fuse == "bn" else "wgrad_dual"
    assert c1.get(key, 0) >= (40 if fuse == "bn" else 50), c1
    for u, u2, v in zip(ref, ref2, got):
        noise = (u2 - u).norm().item()
        assert (v - u).norm().item() <= 4 * noise + 1e-2 * u.norm().item() + 1e-6
