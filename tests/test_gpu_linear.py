"""Weight-streaming skinny GEMMs (conv_igemm.hip, R = S = 1, split-K) vs fp32 PyTorch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # M tokens, K in, N out
    (128, 4096, 4096),
    (128, 4096, 11008),
    (128, 11008, 4096),
    (1, 256, 512),
    (77, 512, 328),
    (300, 1024, 768),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("splits", [-1, 1, 3])
def test_linear_nt_nn_match_fp32(shape, splits):
    from hyperion.ops import _native

    M, K, N = shape
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    y = _native.native().linear_nt(x, w, splits)
    ref = x.float() @ w.float().t()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert (y.float() - ref).norm() <= 1e-2 * ref.norm()
    if N % 64 == 0:
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        dx = _native.native().linear_nn(dy, w, splits)
        refx = dy.float() @ w.float()
        assert dx.shape == (M, K)
        assert (dx.float() - refx).norm() <= 1e-2 * refx.norm()


def test_linear_autograd_matches_reference():
    from hyperion.ops.linear import Linear

    torch.manual_seed(0)
    lin = Linear(512, 1024, bias=True).cuda().to(torch.bfloat16)
    x = torch.randn(4, 32, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = lin(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().float().requires_grad_(True)
    br = lin.bias.detach().float().requires_grad_(True)
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(g.float())
    for a, b in ((y, yr), (x.grad, xr.grad), (lin.weight.grad, wr.grad), (lin.bias.grad, br.grad)):
        assert (a.float() - b).norm() <= 2e-2 * b.norm() + 1e-3


def test_lora_linear_uses_native_base_and_matches():
    from hyperion.ops.lora import lora_linear, lora_linear_reference

    torch.manual_seed(0)
    x = torch.randn(128, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(1024, 512, device="cuda") / 512 ** 0.5).to(torch.bfloat16)
    a = (torch.randn(16, 512, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    bm = (torch.randn(1024, 16, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    y = lora_linear(x, w, None, a, bm, 2.0, 0.0)
    g = torch.randn_like(y)
    y.backward(g)
    xr, ar, br = (t.detach().float().requires_grad_(True) for t in (x, a, bm))
    yr = lora_linear_reference(xr, w.float(), None, ar, br, 2.0)
    yr.backward(g.float())
    for u, v in ((y, yr), (x.grad, xr.grad), (a.grad, ar.grad), (bm.grad, br.grad)):
        assert (u.float() - v).norm() <= 2e-2 * v.norm() + 1e-3


@pytest.mark.parametrize("v_nr", [True, False])
def test_linear_lowrank_epilogue_and_alpha(v_nr):
    from hyperion.ops import _native

    torch.manual_seed(0)
    M, K, N, r = 96, 1024, 512, 16
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    U = torch.randn(M, r, device="cuda").to(torch.bfloat16)
    V = torch.randn(N, r, device="cuda").to(torch.bfloat16) if v_nr else torch.randn(r, N, device="cuda").to(torch.bfloat16)
    mask = (torch.rand(M, N, device="cuda") > 0.3).to(torch.bfloat16)
    y = _native.native().linear_nt(x, w, alpha=0.5, U=U, V=V, v_nr=v_nr, mask=mask, beta=3.0)
    lr = U.float() @ (V.float().t() if v_nr else V.float())
    ref = 0.5 * (x.float() @ w.float().t()) + 3.0 * mask.float() * lr
    assert (y.float() - ref).norm() <= 1e-2 * ref.norm()


def test_lora_dropout_native_matches_reference():
    from hyperion.ops.lora import lora_linear, lora_linear_reference

    torch.manual_seed(0)
    x = torch.randn(2, 64, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(1024, 512, device="cuda") / 512 ** 0.5).to(torch.bfloat16)
    a = (torch.randn(16, 512, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    bm = (torch.randn(1024, 16, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    p, s = 0.1, 2.0
    torch.cuda.manual_seed(11)
    y = lora_linear(x, w, None, a, bm, s, p)
    # the native path draws its mask from the generator's (seed, offset) record: re-seed, take the
    # same record, and materialize the scaled keep mask keep/(1-p) it regenerates in backward
    from hyperion.ops import _native

    torch.cuda.manual_seed(11)
    st = _native.rng_state(x.device)
    keep = _native.native().dropout(x.detach().reshape(128, 512).contiguous(), p, st, mask=True).view(2, 64, 512)
    assert abs((keep != 0).float().mean().item() - (1 - p)) < 0.02
    g = torch.randn_like(y)
    y.backward(g)
    xr, ar, br = (t.detach().float().requires_grad_(True) for t in (x, a, bm))
    yr = lora_linear_reference(xr, w.float(), None, ar, br, s, mask=keep.float())
    yr.backward(g.float())
    for u, v in ((y, yr), (x.grad, xr.grad), (a.grad, ar.grad), (bm.grad, br.grad)):
        assert (u.float() - v).norm() <= 2e-2 * v.norm() + 1e-3


@pytest.mark.parametrize("shape", [(6304, 768), (6304, 3072), (3, 8), (4064, 2304), (128, 11008)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_column_sum_matches_fp64(shape, dtype):
    from hyperion.ops import _native

    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dtype)
    out = _native.native().column_sum(x, torch.float32)
    ref = x.double().sum(0)
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-3)


def test_gelu_linear_act_grads_match_reference():
    from hyperion.ops.linear_act import linear_act

    torch.manual_seed(0)
    x = torch.randn(4, 197, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(512, 256, device="cuda") / 16).to(torch.bfloat16).requires_grad_(True)
    b = (torch.randn(512, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_(True)
    y = linear_act(x, w, b, "gelu")
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.gelu(torch.nn.functional.linear(xr, wr, br))
    yr.backward(g.float())
    for u, v in ((y, yr), (x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (u.float() - v).norm() <= 2e-2 * v.norm() + 1e-3


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("shape", [(6304, 3072), (4064, 2048), (37, 264)])
def test_act_bwd_colsum_matches_autograd(act, shape):
    """Activation backward + bias-gradient column sums in one native pass == aten's
    threshold/gelu backward followed by an fp64 column sum."""
    from hyperion.ops import _native

    torch.manual_seed(0)
    M, N = shape
    z = torch.randn(M, N, device="cuda").bfloat16()
    dh = torch.randn(M, N, device="cuda").bfloat16()
    dy, db = _native.native().act_bwd_colsum(dh, z, 1 if act == "relu" else 2, torch.float32)
    ref = torch.ops.aten.threshold_backward(dh, z, 0) if act == "relu" else torch.ops.aten.gelu_backward(dh, z)
    torch.testing.assert_close(dy.float(), ref.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(db, dy.double().sum(0).float(), atol=1e-2 * M ** 0.5, rtol=1e-3)


@pytest.mark.parametrize("shape", [(6304, 768, 768), (4064, 2048, 256), (4064, 256, 2048), (100, 64, 40)])
def test_linear_wgrad_native_matches_mm(shape):
    """Weight gradients on the native kernels (split-K conv-wgrad kernel for small outputs, the
    tiled MFMA GEMM above) == dyᵀ·x (fp32 reference)."""
    from hyperion.ops import _native, gemm
    from hyperion.ops.linear import WGRAD_NATIVE_MAX, linear_wgrad

    M, K, N = shape
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    _native.reset_counters()
    gemm.set_mode("native")
    try:
        dw = linear_wgrad(dy, x)
    finally:
        gemm.set_mode("auto")
    c = _native.counters()
    small = N * K <= WGRAD_NATIVE_MAX and N % 8 == 0 and K % 64 == 0
    assert c.get("linear_wgrad", 0) == int(small)
    assert c.get("gemm_tn", 0) == int(not small and M % 8 == 0)
    ref = dy.float().t() @ x.float()
    assert (dw.float() - ref).norm() <= 5e-3 * ref.norm()


def test_gelu_backward_fast_erf_within_rounding():
    """act_bwd_colsum's GELU derivative (one exp + an A&S 7.1.26 erf) against the fp64 derivative
    over a dense sweep of pre-activations: within one bf16 rounding of the exact value."""
    import math

    from hyperion.ops import _native

    z64 = torch.linspace(-12, 12, 8192 * 8, dtype=torch.float64)
    z = z64.to("cuda").bfloat16().view(-1, 64)
    dh = torch.ones_like(z)
    dy, _ = _native.native().act_bwd_colsum(dh, z, 2, torch.float32)
    x = z.double()
    ref = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
    err = (dy.double() - ref).abs()
    assert float((err - ref.abs() * 2.0 ** -8 - 1e-6).max()) <= 0, float(err.max())
