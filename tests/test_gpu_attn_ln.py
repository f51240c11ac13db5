"""GPU numerics: flash attention and LayerNorm/RMSNorm kernels vs PyTorch fp32 references."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_attn(q, k, v, causal, kpm=None):
    qf, kf, vf = (x.float().transpose(1, 2) for x in (q, k, v))
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    S = q.shape[1]
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    if kpm is not None:
        s = s.masked_fill(kpm[:, None, None, :].bool(), float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ vf).transpose(1, 2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize(
    "B,S,H,D", [(2, 16, 8, 64), (3, 127, 4, 64), (2, 128, 2, 128), (1, 200, 3, 64), (1, 197, 2, 64), (1, 600, 2, 128)]
)
@pytest.mark.parametrize("causal", [False, True])
def test_attention_fwd_bwd(dtype, B, S, H, D, causal):
    from hyperion.ops.attention import _AttnFn

    torch.manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=dtype) for _ in range(3))
    qr, kr, vr = (x.detach().float().requires_grad_(True) for x in (q, k, v))
    ref = _ref_attn(qr, kr, vr, causal)
    qn, kn, vn = (x.detach().requires_grad_(True) for x in (q, k, v))
    out = _AttnFn.apply(qn, kn, vn, causal, 0.0, None, 1.0 / math.sqrt(D))
    tol = 2e-2 if dtype == torch.bfloat16 else 5e-3
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.to(dtype))
    gt = 5e-2 if dtype == torch.bfloat16 else 1e-2
    for a, b in ((qn, qr), (kn, kr), (vn, vr)):
        torch.testing.assert_close(a.grad.float(), b.grad, atol=gt, rtol=gt)


@pytest.mark.parametrize("S", [128, 300])
def test_attention_bwd_fused_inverse_rope(S):
    """attn_bwd_rope == attn_bwd followed by the inverse RoPE pass (D = 128; direct dQ at S <= 128,
    atomic dQ above)."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(0)
    B, H, D = 2, 4, 128
    q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    scale = 1.0 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, True, scale, 0.0, None, None, True)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(do, q, k, v, o, lse, True, scale, 0.0, None, None, dq, dk, dv)
    C.rope_(dq, dk, None, 10000.0, True)
    dq2, dk2, dv2 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    from hyperion.ops.rope import rope_table

    C.attn_bwd_rope(do, q, k, v, o, lse, True, scale, None, dq2, dk2, dv2, rope_table(S, D, 10000.0, q.device))
    torch.testing.assert_close(dv2, dv, atol=0, rtol=0)
    for a, b in ((dq2, dq), (dk2, dk)):  # one bf16 rounding fewer on the fused path
        err = (a.float() - b.float()).abs().max().item()
        assert err <= 2e-2 * b.float().abs().max().item(), err


@pytest.mark.parametrize("D,causal,p", [(128, True, 0.0), (64, False, 0.0), (64, True, 0.1), (128, False, 0.1)])
def test_attention_bwd_query_split_matches_unsplit(D, causal, p):
    """S <= 128 with few heads: the backward splits each head's query slices over workgroups (dK / dV
    as fp32 partials summed in order).  dQ is computed exactly as unsplit; dK / dV within fp32
    re-association of the same terms."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(0)
    B, S, H = 1, 128, 4
    q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(4))
    scale = 1.0 / math.sqrt(D)
    rng = _native.rng_state(q.device) if p > 0 else None
    o, lse = C.attn_fwd(q, k, v, causal, scale, p, rng, None, True)
    res = []
    try:
        for mode in (1, 0):  # off, automatic (4 heads: split)
            C.attn_set_qsplit(mode)
            g = [torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)]
            C.attn_bwd(do, q, k, v, o, lse, causal, scale, p, rng, None, *g)
            res.append(g)
    finally:
        C.attn_set_qsplit(0)
    torch.testing.assert_close(res[1][0], res[0][0], atol=0, rtol=0)
    for a, b in zip(res[1][1:], res[0][1:]):
        err = (a.float() - b.float()).abs().max().item()
        assert err <= 1e-2 * b.float().abs().max().item() + 1e-6, err


@pytest.mark.parametrize("D,causal", [(128, True), (64, False), (64, True)])
@pytest.mark.parametrize("S", [128, 197])
def test_attention_fwd_one_wave_grid_matches_default(D, causal, S):
    """Few (b, h) pairs: the forward runs one-wave workgroups (32 query rows each) instead of
    4-wave ones — the same per-row arithmetic, so O and the LSE are bit-identical."""
    from hyperion.ops import _native

    C = _native.native()
    torch.manual_seed(0)
    q, k, v = (torch.randn(1, S, 4, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    scale = 1.0 / math.sqrt(D)
    res = []
    try:
        for on in (0, 1):
            C.attn_set_fwd_narrow(on)
            res.append(C.attn_fwd(q, k, v, causal, scale, 0.0, None, None, True))
    finally:
        C.attn_set_fwd_narrow(0)
    torch.testing.assert_close(res[1][0], res[0][0], atol=0, rtol=0)
    torch.testing.assert_close(res[1][1], res[0][1], atol=0, rtol=0)


def test_attention_packed_and_padding_mask():
    from hyperion.ops.attention import attention_packed

    torch.manual_seed(1)
    B, S, H, D = 3, 40, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    kpm = torch.zeros(B, S, dtype=torch.bool, device="cuda")
    kpm[1, 30:] = True
    kpm[2, 5:] = True
    out = attention_packed(qkv, key_padding_mask=kpm)
    qr = qkv.detach().float().requires_grad_(True)
    ref = _ref_attn(qr[:, :, 0], qr[:, :, 1], qr[:, :, 2], False, kpm)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    torch.testing.assert_close(qkv.grad.float(), qr.grad, atol=5e-2, rtol=5e-2)


def test_attention_dropout_statistics_and_determinism():
    from hyperion.ops.attention import _AttnFn

    torch.manual_seed(2)
    B, S, H, D = 2, 64, 2, 64
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    v = torch.ones_like(v)
    o = _AttnFn.apply(q, k, v, False, 0.25, None, 1.0 / 8)
    # with V = 1 the output equals the kept, rescaled probability mass per row: mean ≈ 1
    assert abs(o.float().mean().item() - 1.0) < 0.05


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d", [256, 512, 768, 3072, 4096])
@pytest.mark.parametrize("fused", [False, True])
def test_layernorm(dtype, d, fused):
    from hyperion.ops.layernorm import _LNFn

    torch.manual_seed(0)
    # d > 2048 runs the block-per-row kernels; 2100 rows give them 3 rows per block and a partial last block
    x = torch.randn(2100 if d == 3072 else 37, d, device="cuda", dtype=dtype)
    r = torch.randn_like(x) if fused else None
    w = torch.rand(d, device="cuda") + 0.5
    b = torch.randn(d, device="cuda")
    xr = x.detach().float().clone().requires_grad_(True)
    rr = r.detach().float().clone().requires_grad_(True) if fused else None
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.layer_norm(xr + rr if fused else xr, (d,), wr, br, 1e-5)
    xn = x.detach().clone().requires_grad_(True)
    rn = r.detach().clone().requires_grad_(True) if fused else None
    wn, bn = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yn = _LNFn.apply(xn, rn, wn, bn, 1e-5, False, False)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(yn.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    yr.backward(g)
    yn.backward(g.to(dtype))
    torch.testing.assert_close(xn.grad.float(), xr.grad, atol=tol * 5, rtol=tol * 5)
    torch.testing.assert_close(wn.grad, wr.grad, atol=tol * 20, rtol=tol * 5)
    torch.testing.assert_close(bn.grad, br.grad, atol=tol * 20, rtol=tol * 5)
    if fused:
        torch.testing.assert_close(rn.grad.float(), rr.grad, atol=tol * 5, rtol=tol * 5)


@pytest.mark.parametrize("d", [768, 4096])
@pytest.mark.parametrize("rms", [False, True])
def test_layernorm_bf16_affine(d, rms):
    """bf16 weight / bias (a module cast wholesale to bf16, FSDP mixed precision) read in the kernel;
    dγ / dβ come back in bf16 (no cast kernels around the op)."""
    from hyperion.ops.layernorm import layer_norm

    torch.manual_seed(0)
    x = torch.randn(300, d, device="cuda", dtype=torch.bfloat16)
    w = (torch.rand(d, device="cuda") + 0.5).to(torch.bfloat16)
    b = None if rms else torch.randn(d, device="cuda").to(torch.bfloat16)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    br = None if rms else b.detach().float().requires_grad_(True)
    if rms:
        yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    else:
        yr = F.layer_norm(xr, (d,), wr, br, 1e-5)
    xn, wn = x.detach().requires_grad_(True), w.detach().requires_grad_(True)
    bn = None if rms else b.detach().requires_grad_(True)
    yn = layer_norm(xn, wn, bn, 1e-5, rms=rms)
    torch.testing.assert_close(yn.float(), yr, atol=3e-2, rtol=3e-2)
    g = torch.randn_like(yr)
    yr.backward(g)
    yn.backward(g.to(torch.bfloat16))
    assert wn.grad.dtype == torch.bfloat16
    torch.testing.assert_close(xn.grad.float(), xr.grad, atol=0.15, rtol=0.05)
    torch.testing.assert_close(wn.grad.float(), wr.grad, atol=0.5, rtol=0.05)
    if not rms:
        assert bn.grad.dtype == torch.bfloat16
        torch.testing.assert_close(bn.grad.float(), br.grad, atol=0.5, rtol=0.05)


def test_rmsnorm():
    from hyperion.ops.layernorm import RMSNorm

    torch.manual_seed(0)
    m = RMSNorm(4096).cuda()
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
    x = torch.randn(5, 7, 4096, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = m(x)
    xr = x.detach().float().requires_grad_(True)
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * m.weight
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=5e-2)
