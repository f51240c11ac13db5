"""Hand-written MFMA GEMM (gemm_mfma.hip) vs a plain fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("bk", [32, 64])
@pytest.mark.parametrize("shape", [(128, 128, 64), (256, 384, 512), (1024, 640, 1024), (384, 1152, 4160)])
def test_gemm_nt_matches_fp32(dtype, bk, shape):
    from hyperion.ops import _native

    M, N, K = shape
    if K % bk:
        pytest.skip("K not a multiple of bk")
    torch.manual_seed(0)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(dtype)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(dtype)
    c = _native.native().gemm_nt(a, b, torch.float32, 1.0, bk)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-3 * (K ** 0.5))


def test_gemm_nt_asymmetric_identity():
    # A = I, asymmetric B: catches a transposed C write (cdna guide §3)
    from hyperion.ops import _native

    n = 256
    a = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(n * n, device="cuda", dtype=torch.float32).view(n, n) % 97).to(torch.bfloat16)
    c = _native.native().gemm_nt(a, b, torch.float32, 1.0, 64)
    torch.testing.assert_close(c, b.float().t())


def test_gemm_bf16_out_and_alpha():
    from hyperion.ops import _native

    a = torch.randn(256, 256, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(128, 256, device="cuda", dtype=torch.bfloat16)
    c = _native.native().gemm_nt(a, b, None, 0.5, 64)
    assert c.dtype == torch.bfloat16
    torch.testing.assert_close(c.float(), 0.5 * (a.float() @ b.float().t()), rtol=2e-2, atol=5e-2)


def test_stream_kernels_bandwidth_sane():
    from hyperion.bench.hardware import stream_bandwidth

    r = stream_bandwidth(50_000_000, "add", "hyperion", "proper", repeat=5, warmup=2)
    assert r["Bandwidth (GB/s)"] > 1000  # MI355X HBM3E ≈ 8 TB/s; anything near the MI250X figure is a bug


@pytest.mark.parametrize("shape", [(128, 128, 32), (256, 384, 96), (1024, 512, 2048)])
def test_gemm_f32_nt_matches_fp64(shape):
    """fp32-input MFMA GEMM (gemm_f32.hip): exact fp32 products, fp32 accumulation — error vs fp64
    at the level of a k-ordered fp32 fma chain."""
    from hyperion.ops import _native

    M, N, K = shape
    torch.manual_seed(0)
    a = torch.rand(M, K, device="cuda") * 2 - 1
    b = torch.rand(N, K, device="cuda") * 2 - 1
    c = _native.native().gemm_f32_nt(a, b)
    ref = a.double() @ b.double().t()
    bound = 4e-7 * (a.abs().double() @ b.abs().double().t()) + 1e-30
    assert ((c.double() - ref).abs() <= bound * 8).all()
    assert _native.native().gemm_f32_nt(a, b, out_dtype=torch.bfloat16).dtype == torch.bfloat16
