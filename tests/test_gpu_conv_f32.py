"""fp32 path on the fp32-input MFMA (gemm_f32.hip): the general GEMM (NT / NN / TN, ragged shapes,
split-K, epilogue) and the im2col convolution (ops/conv_f32.py) against fp64 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _native_route(monkeypatch):
    """The numerics tests exercise the native path whatever the per-shape timing would pick."""
    from hyperion.ops import conv_f32

    monkeypatch.setattr(conv_f32, "ROUTE", "native")


def _bound(a, b):
    # a k-ordered fp32 fma chain (or a few of them, summed): error ≲ K·eps·Σ|a||b|; generous factor
    return 8 * 4e-7 * (a.abs() @ b.abs().t()) + 1e-30


@pytest.mark.parametrize("a_tr", [False, True])
@pytest.mark.parametrize("b_tr", [False, True])
@pytest.mark.parametrize("shape", [(128, 128, 32), (100, 200, 36), (1000, 68, 3000), (4, 516, 1028), (257, 129, 260)])
def test_gemm_f32_layouts_match_fp64(a_tr, b_tr, shape):
    from hyperion.ops import _native

    M, N, K = shape
    if (a_tr and M % 4) or (b_tr and N % 4):
        pytest.skip("tr-form extent must be a multiple of 4")
    torch.manual_seed(0)
    a = torch.rand(M, K, device="cuda") * 2 - 1
    b = torch.rand(N, K, device="cuda") * 2 - 1
    A = a.t().contiguous() if a_tr else a
    B = b.t().contiguous() if b_tr else b
    c = _native.native().gemm_f32(A, B, a_tr=a_tr, b_tr=b_tr)
    ref = a.double() @ b.double().t()
    assert ((c.double() - ref).abs() <= _bound(a.double(), b.double())).all()


@pytest.mark.parametrize("splits", [1, 3, 16])
def test_gemm_f32_epilogue_and_splitk(splits):
    from hyperion.ops import _native

    torch.manual_seed(1)
    M, N, K = 300, 260, 1024
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda")
    bias = torch.randn(N, device="cuda")
    old = torch.randn(M, N, device="cuda")
    out = old.clone()
    c = _native.native().gemm_f32(a, b, bias=bias, relu=True, alpha=0.5, beta=1.0, out=out, splits=splits)
    assert c.data_ptr() == out.data_ptr()
    ref = torch.relu(0.5 * (a.double() @ b.double().t()) + bias.double() + old.double())
    torch.testing.assert_close(c.double(), ref, rtol=1e-5, atol=1e-4)


def test_gemm_f32_split_is_deterministic():
    from hyperion.ops import _native

    a = torch.randn(256, 8192, device="cuda")
    b = torch.randn(128, 8192, device="cuda")
    c1 = _native.native().gemm_f32(a, b, splits=8)
    c2 = _native.native().gemm_f32(a, b, splits=8)
    assert torch.equal(c1, c2)


GEOMS = [  # (Cin, Cout, H, R, stride, pad, bias)
    (64, 64, 14, 1, 1, 0, False),
    (64, 128, 14, 3, 1, 1, False),
    (64, 128, 15, 3, 2, 1, True),
    (256, 512, 14, 1, 2, 0, False),
    (3, 64, 32, 7, 2, 3, False),
    (3, 96, 32, 16, 16, 0, True),
]


@pytest.mark.parametrize("geom", GEOMS)
def test_conv2d_f32_fwd_bwd_match_fp64(geom):
    from hyperion.ops import _native
    from hyperion.ops.conv_f32 import Conv2d

    cin, cout, h, r, st, pad, bias = geom
    torch.manual_seed(0)
    conv = Conv2d(cin, cout, r, stride=st, padding=pad, bias=bias).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(2, cin, h, h, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    _native.reset_counters()
    y = conv(x)
    assert _native.counters().get("conv_f32", 0) == 1
    g = torch.randn_like(y)
    y.backward(g)

    xd = x.detach().double().cpu().requires_grad_(True)
    wd = conv.weight.detach().double().cpu().requires_grad_(True)
    bd = conv.bias.detach().double().cpu().requires_grad_(True) if bias else None
    yr = F.conv2d(xd, wd, bd, st, pad)
    yr.backward(g.double().cpu())
    scale = yr.abs().max().item()
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-5, atol=1e-5 * scale)
    torch.testing.assert_close(x.grad.double().cpu(), xd.grad, rtol=1e-5, atol=1e-5 * xd.grad.abs().max().item())
    torch.testing.assert_close(conv.weight.grad.double().cpu(), wd.grad, rtol=1e-5,
                               atol=1e-5 * wd.grad.abs().max().item())
    if bias:
        torch.testing.assert_close(conv.bias.grad.double().cpu(), bd.grad, rtol=1e-5, atol=1e-4)


def test_resnet18_fp32_step_native_matches_vendor():
    """A whole fp32 ResNet-18 forward + backward on the native fp32 convolutions vs the same model on
    F.conv2d (MIOpen): same loss and gradients to fp32 summation-order tolerance."""
    from hyperion.models import resnet18
    from hyperion.ops import _native, conv_f32

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.rand(4, 10, device="cuda")

    def run(native):
        conv_f32.ENABLED = native
        try:
            m.zero_grad(set_to_none=True)
            _native.reset_counters()
            loss = F.mse_loss(m(x), y)
            loss.backward()
            return loss.item(), [p.grad.clone() for p in m.parameters()], _native.counters()
        finally:
            conv_f32.ENABLED = True

    l0, g0, _ = run(False)
    l1, g1, cnt = run(True)
    assert cnt.get("conv_f32", 0) == 20, cnt  # every conv (stem, 16 block convs, 3 downsamples)
    assert abs(l0 - l1) <= 1e-5 * abs(l0)
    for a, b in zip(g0, g1):
        torch.testing.assert_close(b, a, rtol=1e-3, atol=1e-4 * (a.abs().max().item() + 1e-12))


@pytest.mark.parametrize("shape", [(2, 197, 768, 3072), (3, 100, 260, 68)])
def test_linear_f32_native_matches_fp64(shape, monkeypatch):
    """ops/linear_f32.py with the native kernel forced for all three GEMMs vs fp64 F.linear."""
    from hyperion.ops import _native, linear_f32

    monkeypatch.setattr(linear_f32, "_choose", lambda key, native, vendor: native())
    b_, t, fin, fout = shape
    torch.manual_seed(0)
    x = torch.randn(b_, t, fin, device="cuda", requires_grad=True)
    w = (torch.randn(fout, fin, device="cuda") / fin ** 0.5).requires_grad_(True)
    b = torch.randn(fout, device="cuda", requires_grad=True)
    y = linear_f32.linear_f32(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    xd, wd, bd = (t_.detach().double().requires_grad_(True) for t_ in (x, w, b))
    yr = F.linear(xd, wd, bd)
    yr.backward(g.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.double(), xd.grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(w.grad.double(), wd.grad, rtol=1e-5, atol=1e-4 * (t * b_) ** 0.5)
    torch.testing.assert_close(b.grad.double(), bd.grad, rtol=1e-5, atol=1e-4)


def test_conv2d_f32_auto_route_times_both_and_caches(monkeypatch):
    from hyperion.ops import conv_f32

    monkeypatch.setattr(conv_f32, "ROUTE", "auto")
    conv_f32._ROUTE.clear()
    conv = conv_f32.Conv2d(64, 64, 3, padding=1, bias=False).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 64, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y1 = conv(x)
    assert len(conv_f32._ROUTE) == 1
    y2 = conv(x)
    assert len(conv_f32._ROUTE) == 1
    ref = F.conv2d(x.detach(), conv.weight.detach(), None, 1, 1)
    torch.testing.assert_close(y1, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y2, y1)


def test_resnet18_fp32_eval_bn_folded_matches_vendor():
    """Inference with the BN folded into the fp32 GEMM (conv_bn_eval_f32) vs conv + BN on the vendor ops."""
    from hyperion.models import resnet18
    from hyperion.ops import _native, conv_f32

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    for mod in m.modules():  # non-trivial running statistics
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
    m.eval()
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        conv_f32.ENABLED = False
        try:
            ref = m(x)
        finally:
            conv_f32.ENABLED = True
        _native.reset_counters()
        out = m(x)
    assert _native.counters().get("conv_bn_eval_f32", 0) >= 16, _native.counters()
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3 * ref.abs().max().item())
