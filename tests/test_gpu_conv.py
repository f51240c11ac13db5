"""Implicit-GEMM conv (conv_igemm.hip) + fused conv/BN/ReLU vs plain fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # N, C, H, W, K, R, stride, pad
    (2, 64, 14, 14, 64, 3, 1, 1),
    (2, 64, 14, 14, 256, 1, 1, 0),
    (3, 128, 9, 9, 64, 1, 2, 0),
    (2, 128, 15, 15, 128, 3, 2, 1),
    (1, 256, 7, 7, 2048, 1, 1, 0),
    (4, 512, 7, 7, 512, 3, 1, 1),
    (8, 64, 56, 56, 64, 3, 1, 1),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_fwd_and_stats_match_fp32(shape, dtype):
    from hyperion.ops import _native

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).to(dtype).contiguous(
        memory_format=torch.channels_last)
    y, psum, psq = _native.native().conv_fwd(x, w, s, s, p, p, True)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=p)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    yr = y.float()
    torch.testing.assert_close(psum.sum(0).float(), yr.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(psq.sum(0).float(), (yr * yr).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("shape", SHAPES[:5])
@pytest.mark.parametrize("act,res", [(True, False), (True, True), (False, False)])
def test_conv_bn_act_fwd_bwd_match_reference(shape, act, res):
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    _native.reset_counters()
    conv = torch.nn.Conv2d(C, K, R, stride=s, padding=p, bias=False).cuda()
    bn = BatchNormAct2d(K, act=act).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    conv_l = conv.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    P = (H + 2 * p - R) // s + 1
    r = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last) if res else None
    if r is not None:
        r.requires_grad_(True)
    out = conv_bn_act(conv_l, bn, x, r)
    g = torch.randn_like(out)
    out.backward(g)
    cnt = _native.counters()  # the fused kernels ran (a bn(conv(x)) fallback computes the same numbers)
    assert cnt.get("conv_bn_act") == 1 and "conv_bn_act_fallback" not in cnt, cnt
    assert cnt.get("wgrad") == 1 and "wgrad_vendor" not in cnt, cnt
    if s == 1 or R == 1:
        assert "dgrad_vendor" not in cnt, cnt
    # fp32 reference on the CPU: MIOpen's fp32 conv backward segfaults on the host for the
    # N=1, C=256, 7x7, K=2048 1x1 shape (ROCm 7 / torch 2.10; reproduced in isolation), so the
    # oracle does not touch the vendor GPU path at all
    xr = x.detach().float().cpu().requires_grad_(True)
    wr = conv_l.weight.detach().float().cpu().requires_grad_(True)
    rr = r.detach().float().cpu().requires_grad_(True) if res else None
    y = F.conv2d(xr, wr, stride=s, padding=p)
    y = F.batch_norm(y, None, None, bn.weight.detach().cpu(), bn.bias.detach().cpu(), True, 0.1, bn.eps)
    if res:
        y = y + rr
    if act:
        y = F.relu(y)
    y.backward(g.float().cpu())
    assert (out.float().cpu() - y).norm() <= 2e-2 * y.norm() + 1e-3
    assert (x.grad.float().cpu() - xr.grad).norm() <= 3e-2 * xr.grad.norm() + 1e-3
    assert (conv_l.weight.grad.float().cpu() - wr.grad).norm() <= 3e-2 * wr.grad.norm() + 1e-3
    if res:
        assert (r.grad.float().cpu() - rr.grad).norm() <= 3e-2 * rr.grad.norm() + 1e-3


def test_conv_bn_running_stats_updated():
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act

    conv = torch.nn.Conv2d(64, 64, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(64, act=True).cuda()
    x = torch.randn(4, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv_bn_act(conv, bn, x)
    y = F.conv2d(x.float(), conv.weight.float())
    torch.testing.assert_close(bn.running_mean, 0.1 * y.mean((0, 2, 3)), rtol=2e-2, atol=2e-3)
    assert bn.num_batches_tracked.item() + bn._host_batches == 1


WGRAD_SHAPES = SHAPES + [  # N, C, H, W, K, R, stride, pad
    (4, 64, 56, 56, 256, 1, 1, 0),   # layer1 expand (splits, 128x64 tiles)
    (4, 256, 56, 56, 128, 1, 2, 0),  # layer2 downsample 1x1 / 2
    (2, 128, 28, 28, 128, 3, 2, 1),  # stride-2 3x3, 128x128 tiles
    (3, 192, 10, 10, 24, 3, 1, 1),   # K not a multiple of the tile (64x64, masked rows)
]


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_wgrad_matches_fp32(shape, dtype):
    from hyperion.ops import _native

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, P, P, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    dw = _native.native().conv_wgrad(dy, x, R, R, s, s, p, p)
    assert dw.shape == (K, C, R, R) and dw.dtype == dtype and dw.is_contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float().cpu(), (K, C, R, R), dy.float().cpu(), stride=s, padding=p)
    err = (dw.float().cpu() - ref).norm() / ref.norm()
    assert err < 1e-2, f"rel err {err:.3e}"


@pytest.mark.parametrize("cfg", [(64, 64, 1, 2), (64, 64, 7, 3), (128, 128, 3, 2), (128, 64, 5, 4),
                                 (64, 128, 2, 2), (128, 128, 1, 3),
                                 # | 32: 128-pixel stages (dense kernel), | 16: dense shapes on the general kernel
                                 (64, 64, 3, 2 | 32), (128, 64, 2, 3 | 32), (128, 128, 5, 2 | 32), (64, 64, 2, 2 | 16)])
@pytest.mark.parametrize("shape", [(3, 256, 9, 9, 128, 1, 1, 0),    # dense 1x1, M = 243 (tail stage)
                                   (2, 128, 13, 13, 192, 3, 1, 1),  # gathered 3x3, K % 128 != 0
                                   (5, 128, 11, 11, 128, 1, 2, 0)])  # strided 1x1, several images per stage
def test_conv_wgrad_tiles_splits_stages(shape, cfg):
    """Every tile / split / LDS-ring variant of conv_wgrad.hip (the automatic plan picks among
    them) against the fp32 reference, on dense and gathered inputs with partial stages."""
    from hyperion.ops import _native

    C_ = _native.native()
    N, C, H, W, K, R, s, p = shape
    bm, bn, splits, nb = cfg
    torch.manual_seed(0)
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float().cpu(), (K, C, R, R), dy.float().cpu(), stride=s, padding=p)
    C_.conv_set_stages(0, nb)
    try:
        dw = C_.conv_wgrad(dy, x, R, R, s, s, p, p, bm, bn, splits)
    finally:
        C_.conv_set_stages(0, 0)
    err = (dw.float().cpu() - ref).norm() / ref.norm()
    assert err < 1e-2, f"rel err {err:.3e}"


@pytest.mark.parametrize("shape", [s for s in WGRAD_SHAPES if s[6] == 1 and s[4] % 64 == 0])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_conv_dgrad_matches_fp32(shape, dtype):
    from hyperion.ops import _native

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    P = (H + 2 * p - R) // s + 1
    w = (torch.randn(K, C, R, R, device="cuda") / (K * R * R) ** 0.5).to(dtype).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, K, P, P, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    dx = _native.native().conv_dgrad(dy, w, p, p)
    assert dx.shape == (N, C, H, W) and dx.is_contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.float().cpu(), dy.float().cpu(), stride=s, padding=p)
    err = (dx.float().cpu() - ref).norm() / ref.norm()
    assert err < 1e-2, f"rel err {err:.3e}"


@pytest.mark.parametrize("shape", [(32, 512, 7, 7, 512, 3, 1, 1), (32, 2048, 7, 7, 512, 1, 1, 0),
                                   (32, 256, 14, 14, 256, 3, 1, 1), (5, 128, 9, 9, 72, 3, 1, 1)])
@pytest.mark.parametrize("splits", [1, 2, 5, -1])
def test_conv_splitk_fwd_stats_and_dgrad(shape, splits):
    """Split-K forward (BN statistics from the split-K reduce) and split-K dgrad vs fp32."""
    from hyperion.ops import _native

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    y, psum, psq = _native.native().conv_fwd(x, w, s, s, p, p, True, splits=splits)
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=p)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    yr = y.float()
    torch.testing.assert_close(psum.sum(0).float(), yr.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(psq.sum(0).float(), (yr * yr).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    if K % 64 == 0:
        dy = torch.randn(N, K, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        dx = _native.native().conv_dgrad(dy, w, p, p, splits=splits)
        dref = torch.nn.grad.conv2d_input((N, C, H, W), w.float(), dy.float(), stride=1, padding=p)
        err = (dx.float() - dref).norm() / dref.norm()
        assert err < 1e-2, f"rel err {err:.3e}"


@pytest.mark.parametrize("shape,splits", [((4, 256, 14, 14, 64, 1, 1, 0), 1), ((8, 64, 14, 14, 64, 3, 1, 1), 1),
                                          ((4, 512, 7, 7, 512, 3, 1, 1), 3)])
def test_conv_dgrad_addend_is_exact_separate_add(shape, splits):
    """dgrad with the fused addend == dgrad followed by a bf16 add, bit for bit."""
    from hyperion.ops import _native

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    w = (torch.randn(K, C, R, R, device="cuda") / (K * R * R) ** 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    add = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    C_ = _native.native()
    ref = C_.conv_dgrad(dy, w, p, p, splits=splits) + add
    got = C_.conv_dgrad(dy, w, p, p, splits=splits, addend=add)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("block", ["bottleneck", "basic"])
def test_shortcut_grad_fusion_matches_autograd_add(block):
    """ResNet blocks with the identity-shortcut gradient fused into conv1's dgrad produce the
    same gradients as autograd's separate add (bitwise)."""
    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import BasicBlock, Bottleneck
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = (Bottleneck(256, 64) if block == "bottleneck" else BasicBlock(64, 64)).cuda()
    m = m.to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    cin = 256 if block == "bottleneck" else 64
    x0 = torch.randn(8, cin, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, cin, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)

    def run(fuse):
        hconv.FUSE_SHORTCUT_GRAD = fuse
        hconv.FUSE_BN_BACKWARD = False  # bitwise A/B of the shortcut fusion alone (see test_bn_backward_fusion)
        try:
            for p in m.parameters():
                p.grad = None
            x = x0.clone().requires_grad_(True)
            m(x).backward(gy)
            return [x.grad.clone()] + [p.grad.clone() for p in m.parameters()]
        finally:
            hconv.FUSE_SHORTCUT_GRAD = True
            hconv.FUSE_BN_BACKWARD = True

    a, b = run(False), run(True)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("shape", [(4, 256, 14, 14, 2, 2), (2, 64, 7, 9, 2, 2), (3, 128, 8, 8, 1, 1), (2, 8, 6, 6, 3, 2)])
@pytest.mark.parametrize("with_add", [False, True])
def test_upsample_add_matches_reference(shape, with_add):
    """comp scattered to every s-th pixel (+ addend) == zeros / strided assign / bf16 add, bit for bit."""
    from hyperion.ops import _native

    N, C, H, W, sh, sw = shape
    P, Q = (H - 1) // sh + 1, (W - 1) // sw + 1
    torch.manual_seed(0)
    comp = torch.randn(N, C, P, Q, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    add = (torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
           if with_add else None)
    ref = torch.zeros(N, C, H, W, device="cuda", dtype=torch.bfloat16)
    ref[:, :, ::sh, ::sw] = comp
    if with_add:
        ref = ref + add
    got = _native.native().upsample_add(comp, add, H, W, sh, sw)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("shape", [(4, 256, 28, 28, 512), (8, 1024, 14, 14, 2048), (2, 64, 7, 7, 128)])
def test_strided_1x1_dgrad_matches_fp32(shape):
    """1x1 stride-2 data gradient (DGRAD GEMM on the output grid + scatter) vs the fp32 reference."""
    from hyperion.ops.conv import _dgrad

    N, C, H, W, K = shape
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 1, 1, device="cuda") / C ** 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = torch.randn(N, K, P, Q, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dx = _dgrad(dy, x, w, (2, 2), (0, 0))
    dref = torch.nn.grad.conv2d_input((N, C, H, W), w.float(), dy.float(), stride=2, padding=0)
    err = (dx.float() - dref).norm() / dref.norm()
    assert err < 1e-2, f"rel err {err:.3e}"
    assert torch.all(dx[:, :, 1::2, :] == 0) and torch.all(dx[:, :, :, 1::2] == 0)


@pytest.mark.parametrize("block", ["bottleneck_s2", "bottleneck_s1", "basic_s2"])
def test_downsample_branch_grad_fusion_matches_autograd_add(block):
    """Downsampling blocks with the two data gradients of the block input summed in-kernel
    (BranchSumLink) produce the same gradients as autograd's separate add (bitwise)."""
    import torch.nn as nn

    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import BasicBlock, Bottleneck, conv1x1
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    if block == "bottleneck_s2":
        cin, cout, s, HW = 256, 512, 2, 14
        m = Bottleneck(cin, 128, 2, nn.Sequential(conv1x1(cin, cout, 2), BatchNormAct2d(cout)))
    elif block == "bottleneck_s1":
        cin, cout, s, HW = 64, 256, 1, 14
        m = Bottleneck(cin, 64, 1, nn.Sequential(conv1x1(cin, cout, 1), BatchNormAct2d(cout)))
    else:
        cin, cout, s, HW = 64, 128, 2, 14
        m = BasicBlock(cin, 128, 2, nn.Sequential(conv1x1(cin, cout, 2), BatchNormAct2d(cout)))
    m = m.cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, cin, HW, HW, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, cout, HW // s, HW // s, device="cuda").bfloat16().contiguous(
        memory_format=torch.channels_last)

    def run(fuse):
        hconv.FUSE_SHORTCUT_GRAD = fuse
        hconv.FUSE_BN_BACKWARD = False  # bitwise A/B of the shortcut fusion alone (see test_bn_backward_fusion)
        try:
            for p in m.parameters():
                p.grad = None
            x = x0.clone().requires_grad_(True)
            m(x).backward(gy)
            return [x.grad.clone()] + [p.grad.clone() for p in m.parameters()]
        finally:
            hconv.FUSE_SHORTCUT_GRAD = True
            hconv.FUSE_BN_BACKWARD = True

    # the strided 3x3 conv's data gradient is MIOpen's: pin its deterministic algorithm
    det, bench = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        a, b = run(False), run(True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bench
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("block", ["bottleneck_s2", "bottleneck_id"])
def test_partial_backward_with_gradient_links(block):
    """A partial ``autograd.grad`` (retain_graph) that reaches only one consumer of a block input
    must not park a gradient for a partner that never runs: the following full backward still
    matches the unfused gradients bitwise (BranchSumLink / ResidualLink staleness)."""
    import torch.nn as nn

    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import Bottleneck, conv1x1
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    if block == "bottleneck_s2":
        cin, cout, s = 256, 512, 2
        m = Bottleneck(cin, 128, 2, nn.Sequential(conv1x1(cin, cout, 2), BatchNormAct2d(cout)))
        probe = m.downsample[0].weight
    else:
        cin, cout, s = 256, 256, 1
        m = Bottleneck(cin, 64)
        probe = m.conv3.weight
    m = m.cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, cin, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, cout, 14 // s, 14 // s, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)

    def run(fuse, partial):
        hconv.FUSE_SHORTCUT_GRAD = fuse
        hconv.FUSE_BN_BACKWARD = False  # bitwise A/B of the shortcut fusion alone (see test_bn_backward_fusion)
        try:
            x = x0.clone().requires_grad_(True)
            out = m(x)
            if partial:  # reaches the probe's consumer only
                torch.autograd.grad(out, [probe], gy, retain_graph=True)
            return torch.autograd.grad(out, [x], gy)[0]
        finally:
            hconv.FUSE_SHORTCUT_GRAD = True
            hconv.FUSE_BN_BACKWARD = True

    det, bench = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        ref = run(False, False)
        got = run(True, True)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det, bench
    assert torch.equal(ref, got)


@pytest.mark.parametrize("arch", ["resnet50", "resnet18"])
def test_bn_backward_fusion_matches_unfused(arch, monkeypatch):
    """The BN-backward reduce computed in the consuming conv's dgrad epilogue (BNGradLink: dz =
    dX·mask, Σdz, Σdz·x into the producer's sums) vs the separate reduce pass: both bf16 paths
    are as close to an fp32 reference of the same network (torch ops, same weights) as each other,
    and the fused path actually ran (dispatch counter)."""
    import copy

    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import resnet18, resnet50
    from hyperion.ops import _native
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m32 = (resnet50 if arch == "resnet50" else resnet18)(num_classes=16).cuda().to(memory_format=torch.channels_last)
    m = copy.deepcopy(m32)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(4, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(4, 16, device="cuda").bfloat16()

    modes = hconv.FUSE_BN_MODES
    hconv.FUSE_BN_MODES = {0, 1, 2}  # every producer kind

    def run(fuse):
        hconv.FUSE_BN_BACKWARD = fuse
        try:
            for p in m.parameters():
                p.grad = None
            _native.reset_counters()
            x = x0.clone().requires_grad_(True)
            m(x).backward(gy)
            torch.cuda.synchronize()
            return [x.grad.float().clone()] + [p.grad.float().clone() for p in m.parameters()], _native.counters()
        finally:
            hconv.FUSE_BN_BACKWARD = True

    try:
        a, ca = run(False)
        b, cb = run(True)
    finally:
        hconv.FUSE_BN_MODES = modes
    assert ca.get("dgrad_bn_fused", 0) == 0
    assert cb.get("dgrad_bn_fused", 0) >= (20 if arch == "resnet50" else 5), cb
    monkeypatch.setenv("HYPERION_KERNELS", "torch")
    xr = x0.float().requires_grad_(True)
    m32(xr).backward(gy.float())
    ref = [xr.grad] + [p.grad for p in m32.parameters()]

    def rel(u, r):
        return ((u - r).norm() / (r.norm() + 1e-12)).item()

    ea = [rel(u, r) for u, r in zip(a, ref)]
    eb = [rel(v, r) for v, r in zip(b, ref)]
    ma, mb = sorted(ea)[len(ea) // 2], sorted(eb)[len(eb) // 2]
    print(f"vs fp32: unfused median {ma:.2e} max {max(ea):.2e}; fused median {mb:.2e} max {max(eb):.2e}")
    assert mb <= 1.25 * ma + 1e-3, (ma, mb)
    assert max(eb) <= 1.5 * max(ea) + 1e-2, (max(ea), max(eb))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_autocast_resnet18_runs_native_kernels(dt, monkeypatch):
    """The reference AMP trainers (C19 / C23 / C24) run under torch.autocast with fp32 weights:
    conv_bn_act casts x / W to the autocast dtype and takes the fused kernels (dispatch counters),
    and its gradients are as close to the fp32 network's as torch's own autocast path is.  (A
    random-init ResNet at CIFAR size is chaotic in its backward — bf16/fp16 round-off alone moves
    the stem gradients ~40% off fp32 for torch AND native — so the check is relative to torch.)"""
    import copy

    from hyperion.models.resnet import resnet18
    from hyperion.ops import _native

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    m32 = copy.deepcopy(m)
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")

    def run(model, amp):
        for p in model.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=dt, enabled=amp):
            loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach().float(), [p.grad.float().clone() for p in model.parameters()]

    _native.reset_counters()
    l1, g1 = run(m, True)
    cnt = _native.counters()
    assert cnt.get("conv_bn_act", 0) >= 18 and cnt.get("wgrad", 0) >= 18, cnt
    monkeypatch.setenv("HYPERION_KERNELS", "torch")
    l2, g2 = run(m, True)
    l3, g3 = run(m32, False)

    def rel(u, r):
        return ((u - r).norm() / (r.norm() + 1e-12)).item()

    en = sorted(rel(a, r) for a, r in zip(g1, g3))
    et = sorted(rel(b, r) for b, r in zip(g2, g3))
    print(f"vs fp32: native median {en[len(en) // 2]:.2e}, torch autocast median {et[len(et) // 2]:.2e}")
    torch.testing.assert_close(l1, l3, rtol=2e-2, atol=2e-2)
    assert en[len(en) // 2] <= 1.25 * et[len(et) // 2] + 1e-3
    assert rel(g1[-2], g3[-2]) < 5e-2  # fc.weight: before the chaotic depth


@pytest.mark.parametrize("shape", [(8, 64, 16, 16, 64, 3, 1, 1), (8, 128, 8, 8, 256, 1, 1, 0), (32, 512, 1, 1, 512, 3, 1, 1),
                                   (4, 256, 14, 14, 512, 1, 2, 0), (32, 256, 2, 2, 256, 3, 1, 1)])
@pytest.mark.parametrize("act,use_res", [(True, False), (True, True), (False, False)])
def test_conv_bn_eval_fused_matches_composition(shape, act, use_res):
    """Eval-mode conv -> BN(running stats) -> (+res) -> (ReLU) in one launch (BN folded into the
    conv epilogue, split-K reduce included) == the fp32 composition to bf16 rounding."""
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act

    N, C, H, W, K, R, s, p = shape
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(C, K, R, stride=s, padding=p, bias=False).cuda()
    bn = BatchNormAct2d(K, act=act).cuda()
    with torch.no_grad():
        bn.running_mean.normal_(0, 0.3)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.2)
    conv = conv.to(torch.bfloat16).to(memory_format=torch.channels_last)
    bn.eval()
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    P = (H + 2 * p - R) // s + 1
    res = (torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
           if use_res else None)
    _native.reset_counters()
    with torch.no_grad():
        got = conv_bn_act(conv, bn, x, residual=res)
    assert _native.counters().get("conv_bn_eval", 0) == 1
    with torch.no_grad():
        yr = torch.nn.functional.conv2d(x.float(), conv.weight.float(), stride=s, padding=p)
        yr = (yr - bn.running_mean.view(1, -1, 1, 1)) * torch.rsqrt(bn.running_var.view(1, -1, 1, 1) + bn.eps)
        yr = yr * bn.weight.view(1, -1, 1, 1) + bn.bias.view(1, -1, 1, 1)
        if use_res:
            yr = yr + res.float()
        if act:
            yr = torch.relu(yr)
    assert got.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(got.float(), yr, atol=3e-2, rtol=3e-2)


def test_resnet18_inference_fused_path():
    """ResNet-18 CIFAR inference (the C32 fusion benchmark's config: eval, no_grad, bf16 autocast,
    fp32 weights): every 64-channel-aligned conv+BN(+res)(+ReLU) is one fused launch, and the
    logits match PyTorch's eager path."""
    from hyperion.models.resnet import resnet18
    from hyperion.ops import _native

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last).eval()
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    _native.reset_counters()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        got = m(x).float()
    assert _native.counters().get("conv_bn_eval", 0) >= 18, _native.counters()
    import os
    os.environ["HYPERION_KERNELS"] = "torch"
    try:
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            ref = m(x).float()
    finally:
        os.environ.pop("HYPERION_KERNELS")
    torch.testing.assert_close(got, ref, atol=5e-2, rtol=5e-2)


def test_resnet_training_mode_forward_under_no_grad():
    """A train-mode forward with autograd off (e.g. a benchmark's no-grad timing pass) takes the
    fused training kernels without building gradient links (regression: weakref to a None grad_fn)."""
    from hyperion.models.resnet import resnet50
    from hyperion.train.amp import cast_for_compute

    m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x = torch.randn(2, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = m(x)
    assert torch.isfinite(y.float()).all()


@pytest.mark.parametrize("accumulate", [False, True])
def test_deferred_wgrad_reduce_is_exact(accumulate):
    """Weight-gradient split-K reduces chained into the next conv_wgrad launch (ops/conv.py
    DEFER_WGRAD_REDUCE) give the gradients of the standalone reduce kernels (two bottleneck blocks);
    with gradients already allocated (accumulation: AccumulateGrad reads dW at once) nothing is
    deferred."""
    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import Bottleneck
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = torch.nn.Sequential(Bottleneck(256, 64), Bottleneck(256, 64)).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, 256, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 256, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)

    def run(defer):
        hconv.DEFER_WGRAD_REDUCE = defer
        hconv.FUSE_BN_BACKWARD = False
        try:
            for p in m.parameters():
                p.grad = torch.ones_like(p) if accumulate else None
            m(x0).backward(gy)
            torch.cuda.synchronize()
            assert not hconv._defer_state["pending"]
            return [p.grad.float().clone() for p in m.parameters()]
        finally:
            hconv.DEFER_WGRAD_REDUCE = True
            hconv.FUSE_BN_BACKWARD = True

    # the BN statistics' fp64 atomics make two runs of either path differ in the last bits: compare
    # against that run-to-run noise (a wrong or missing reduce is off by O(|grad|))
    ref, ref2, got = run(False), run(False), run(True)
    for u, u2, v in zip(ref, ref2, got):
        assert (v - u).norm().item() <= 4 * (u2 - u).norm().item() + 1e-3 * u.norm().item() + 1e-6


def test_deferred_wgrad_reduce_resnet50_matches():
    """The chained reduces across a whole ResNet-50 backward: gradients agree with the standalone
    reduce path to the run-to-run noise of the BN statistics atomics."""
    import hyperion.ops.conv as hconv
    from hyperion.models.resnet import resnet50
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = resnet50(num_classes=16).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 16, device="cuda").bfloat16()

    def run(defer):
        hconv.DEFER_WGRAD_REDUCE = defer
        try:
            for p in m.parameters():
                p.grad = None
            m(x0).backward(gy)
            torch.cuda.synchronize()
            return [p.grad.float().clone() for p in m.parameters()]
        finally:
            hconv.DEFER_WGRAD_REDUCE = True

    ref, ref2, got = run(False), run(False), run(True)
    for u, u2, v in zip(ref, ref2, got):
        noise = (u2 - u).norm().item()
        assert (v - u).norm().item() <= 4 * noise + 1e-2 * u.norm().item() + 1e-6
