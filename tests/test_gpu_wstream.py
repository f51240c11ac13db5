"""Numerics of the weight-streaming GEMM (csrc/kernels/wstream.hip) against fp32 torch references.

The kernel serves the few-token projections of the Llama LoRA step (reference
``02_development/distributed_utils.py:463-476``): NT (``x Wᵀ``, the forward) and NN (``x W``, the
data gradient with W read in its stored [out, in] layout), with fp32 partial slabs summed by
``ws_reduce`` (+ alpha, addend, rank-r LoRA term).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from hyperion.ops import _native

    return _native.native()


def _ref(x, w, nn):
    return x.float() @ (w.float() if nn else w.float().t())


def _close(y, ref, rel=2e-2):
    err = (y.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= rel * scale, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("nn", [False, True])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (128, 1024, 11008), (17, 512, 1024), (64, 768, 384),
                                   (200, 320, 512), (1, 256, 256), (127, 12288 // 4, 4096)])
def test_ws_linear_matches_fp32(M, N, K, nn):
    if nn and N % 64:
        pytest.skip("NN needs N % 64")
    torch.manual_seed(0)
    C = _C()
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") if nn else torch.randn(N, K, device="cuda")).mul_(0.05).bfloat16()
    y = C.ws_linear(x, w, nn=nn)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    _close(y, _ref(x, w, nn))


@pytest.mark.parametrize("nn", [False, True])
@pytest.mark.parametrize("mf,kr,G,nf", [(8, 512, 32, 2), (8, 256, 8, 1), (4, 1024, 5, 4), (2, 2048, 3, 2),
                                        (8, 128, 64, 4)])
def test_ws_plans_agree(mf, kr, G, nf, nn):
    """Every (m-block, slice, column-group, fragments-per-chunk) plan gives the same sums."""
    torch.manual_seed(1)
    C = _C()
    M, N, K = 100, 1024, 2048
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") if nn else torch.randn(N, K, device="cuda")).mul_(0.05).bfloat16()
    y = C.ws_linear(x, w, nn=nn, mf=mf, kr=kr, G=G, nf=nf)
    _close(y, _ref(x, w, nn))


def test_ws_strided_operands_and_f16():
    """Row-strided views (a column block of a concatenated weight / activation) and fp16."""
    torch.manual_seed(2)
    C = _C()
    xb = torch.randn(64, 1024 + 256, device="cuda", dtype=torch.float16)
    wb = (torch.randn(3 * 256, 1024 + 128, device="cuda") * 0.05).half()
    x, w = xb[:, :1024], wb[256:512, :1024]
    y = C.ws_linear(x, w)
    _close(y, _ref(x, w, False))


def test_ws_reduce_epilogue_rank_r_and_addend():
    """out = alpha Σ + beta addend + uscale Σ_r U[m, seg r + rr] V[n, rr] (the LoRA up-projection)."""
    torch.manual_seed(3)
    C = _C()
    M, N, K, r, segw = 128, 3 * 512, 1024, 16, 512
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    U = torch.randn(M, 3 * r, device="cuda")
    V = (torch.randn(N, r, device="cuda") * 0.1).bfloat16()
    add = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    part, S, MFtot = C.ws_gemm_part(x, w)
    y = C.ws_reduce(part, M, N, S, MFtot, False, torch.bfloat16, alpha=0.5, addend=add, beta=2.0, U=U, V=V,
                    segw=segw, uscale=1.5)
    ref = 0.5 * _ref(x, w, False) + 2.0 * add.float()
    for sgm in range(3):
        cols = slice(sgm * segw, (sgm + 1) * segw)
        ref[:, cols] += 1.5 * U[:, sgm * r:(sgm + 1) * r] @ V[cols].float().t()
    _close(y, ref)


def test_ws_deterministic():
    torch.manual_seed(4)
    C = _C()
    x = torch.randn(128, 4096, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(4096, 1024, device="cuda") * 0.05).bfloat16()
    a = C.ws_linear(x, w, nn=True)
    b = C.ws_linear(x, w, nn=True)
    assert torch.equal(a, b)


@pytest.mark.parametrize("nn", [False, True])
def test_ws_bf16_slabs_match_fp32_slabs(nn):
    """bf16 partial slabs (the Llama layer's default): same sums as the fp32 slabs within bf16 output
    rounding, through both the plain reduce and the fused epilogue."""
    torch.manual_seed(3)
    C = _C()
    M, N, K = 128, 1024, 8192
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") if nn else torch.randn(N, K, device="cuda")).mul_(0.05).bfloat16()
    p32, S, MFt = C.ws_gemm_part(x, w, nn=nn)
    p16, S2, MFt2 = C.ws_gemm_part(x, w, nn=nn, slab16=True)
    assert p16.dtype == torch.bfloat16 and (S, MFt) == (S2, MFt2) and S > 1
    ref = _ref(x, w, nn)
    y32 = C.ws_reduce(p32, M, N, S, MFt, nn, torch.bfloat16)
    y16 = C.ws_reduce(p16, M, N, S, MFt, nn, torch.bfloat16)
    _close(y32, ref)
    _close(y16, ref)
    _close(y16, y32.float(), rel=1e-2)
    e16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C.ws_epilogue(p16, S, MFt, M, N, 0, e16, nn=nn)
    _close(e16, y16.float(), rel=1e-2)
