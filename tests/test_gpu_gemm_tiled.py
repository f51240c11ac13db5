"""Deep-pipelined MFMA GEMM (gemm_tiles.hip) vs a plain fp32 PyTorch reference: NT / NN / TN
operand layouts, every tile config, split-K, ragged M/N/K, and the fused epilogues (bias, ReLU,
GELU with the pre-activation output, residual, alpha/beta accumulate)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from hyperion.ops import _native

    return _native.native()


def _rand(*shape, dtype=torch.bfloat16):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(dtype)


def _operands(M, N, K, a_tr, b_tr, dtype):
    a = _rand(K, M, dtype=dtype) if a_tr else _rand(M, K, dtype=dtype)
    b = _rand(K, N, dtype=dtype) if b_tr else _rand(N, K, dtype=dtype)
    af = a.float().t() if a_tr else a.float()
    bf = b.float().t() if b_tr else b.float()
    return a, b, af @ bf.t()


TILE_SHAPES = {0: (256, 256), 1: (256, 128), 2: (128, 128), 4: (64, 64), 5: (128, 64), 6: (64, 128), 7: (192, 128),
               # ping-pong tiles (gemm_pp_k: two 4-wave groups alternating MFMA / load intervals)
               8: (256, 256), 9: (256, 128), 10: (128, 256), 11: (128, 128), 12: (256, 256)}


@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
@pytest.mark.parametrize("tile", [0, 1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 12])
@pytest.mark.parametrize("shape", [(256, 256, 64), (392, 776, 200), (1000, 264, 1032), (2032, 768, 768)])
def test_gemm_layouts_tiles_fp32_out(layout, tile, shape):
    M, N, K = shape
    a_tr, b_tr = layout[0] == "t", layout[1] == "n"
    torch.manual_seed(0)
    a, b, ref = _operands(M, N, K, a_tr, b_tr, torch.bfloat16)
    bm, bn = TILE_SHAPES[tile]
    if (a_tr and bm % 128) or (b_tr and bn % 128):
        with pytest.raises(RuntimeError):  # a transposed operand needs 128-column tile sides
            _C().gemm(a, b, a_tr=a_tr, b_tr=b_tr, out_dtype=torch.float32, tile=tile, splits=1)
        return
    c = _C().gemm(a, b, a_tr=a_tr, b_tr=b_tr, out_dtype=torch.float32, tile=tile, splits=1)
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)


@pytest.mark.parametrize("splits", [2, 3, 7])
@pytest.mark.parametrize("layout", ["nt", "tn"])
def test_gemm_split_k(splits, layout):
    M, N, K = 512, 384, 3072
    a_tr, b_tr = layout[0] == "t", layout[1] == "n"
    torch.manual_seed(1)
    a, b, ref = _operands(M, N, K, a_tr, b_tr, torch.bfloat16)
    c = _C().gemm(a, b, a_tr=a_tr, b_tr=b_tr, out_dtype=torch.float32, tile=2, splits=splits)
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)


def test_gemm_fp16_and_identity():
    # A = I with an asymmetric B catches a transposed C write (cdna guide §3)
    n = 256
    a = torch.eye(n, device="cuda", dtype=torch.float16)
    b = (torch.arange(n * n, device="cuda", dtype=torch.float32).view(n, n) % 97).to(torch.float16)
    for tile in (0, 1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 12):
        c = _C().gemm(a, b, out_dtype=torch.float32, tile=tile, splits=1)
        torch.testing.assert_close(c, b.float().t())


@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_gemm_epilogue_bias_act_aux_residual(act):
    M, N, K = 6304 // 8, 768, 768
    torch.manual_seed(2)
    x, w, ref = _operands(M, N, K, False, False, torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    res = _rand(M, N)
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act else None
    y = _C().gemm(x, w, bias=bias, act=act, aux=aux, residual=res)
    z = (ref + bias).bfloat16().float()
    if act == 1:
        h = F.relu(z)
    elif act == 2:
        h = F.gelu(z)
    elif act == 3:
        h = F.gelu(z, approximate="tanh")
    else:
        h = ref + bias
    want = h.bfloat16().float() + res.float()
    torch.testing.assert_close(y.float(), want, rtol=2e-2, atol=2e-2)
    if act:
        torch.testing.assert_close(aux.float(), z, rtol=1e-2, atol=1e-2)


def test_gemm_alpha_beta_accumulate_fp32():
    # weight-gradient accumulation: out = alpha * A^T B + beta * out
    M, N, K = 768, 3072, 4064
    torch.manual_seed(3)
    dy, x, ref = _operands(M, N, K, True, True, torch.bfloat16)
    out = torch.randn(M, N, device="cuda")
    want = 0.5 * ref + out
    c = _C().gemm(dy, x, a_tr=True, b_tr=True, out=out, alpha=0.5, beta=1.0)
    assert c.data_ptr() == out.data_ptr()
    torch.testing.assert_close(out, want, rtol=1e-4, atol=2e-3 * K ** 0.5)


def test_gemm_strided_operands_and_auto_plan():
    # row-strided views (e.g. q/k/v column slices) and the automatic tile / split plan
    torch.manual_seed(4)
    big = _rand(1000, 2304)
    x = big[:, 768:1536]
    w = _rand(512, 768)
    c = _C().gemm(x, w)
    torch.testing.assert_close(c.float(), x.float() @ w.float().t(), rtol=2e-2, atol=5e-2)
    for shape in [(6304, 768, 3072), (6304, 3072, 768), (768, 3072, 6304), (8192, 8192, 8192), (128, 4096, 4096)]:
        t, s = _C().gemm_plan(*shape)
        assert 0 <= t <= 7 and t != 3 and s >= 1


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("splits", [2, 5])
def test_split_k_last_arriver_matches_separate_reduce(layout, splits):
    """Split-K reduced by the last-arriving workgroup of each tile (arrival counters, write-through
    slabs) == the separate gemm_splitk_epi_k reduce, bitwise (same slice order), with the fused
    bias + GELU + aux epilogue; repeated launches reuse the self-resetting counters."""
    M, N, K = 1000, 776, 2048
    a_tr, b_tr = layout[0] == "t", layout[1] == "n"
    torch.manual_seed(2)
    a, b, ref = _operands(M, N, K, a_tr, b_tr, torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    C = _C()
    outs = {}
    try:
        for mode in (0, 1):
            C.gemm_set_splitk_inkernel(mode)
            aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            rs = [C.gemm(a, b, a_tr=a_tr, b_tr=b_tr, bias=bias, act=2, aux=aux, tile=2, splits=splits) for _ in range(3)]
            outs[mode] = (rs, aux.clone())
    finally:
        C.gemm_set_splitk_inkernel(0)
    torch.cuda.synchronize()
    for r in outs[1][0]:
        assert torch.equal(r, outs[0][0][0])
    assert torch.equal(outs[1][1], outs[0][1])
    z = ref + bias
    torch.testing.assert_close(outs[1][1].float(), z, rtol=2e-2, atol=2e-2 * K ** 0.5)


def test_split_k_last_arriver_under_graph_capture():
    """A captured split-K GEMM takes its own counter range; replays give the eager result."""
    M, N, K = 512, 384, 3072
    torch.manual_seed(3)
    a, b, ref = _operands(M, N, K, False, False, torch.bfloat16)
    C = _C()
    C.gemm_set_splitk_inkernel(1)
    try:
        _captured_split_k(C, a, b, ref, K)
    finally:
        C.gemm_set_splitk_inkernel(0)


def _captured_split_k(C, a, b, ref, K):
    eager = C.gemm(a, b, out_dtype=torch.float32, tile=2, splits=4)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        C.gemm(a, b, out_dtype=torch.float32, tile=2, splits=4)  # warm-up off the capture
        with torch.cuda.graph(g):
            out = C.gemm(a, b, out_dtype=torch.float32, tile=2, splits=4)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
    torch.testing.assert_close(eager, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)


@pytest.mark.parametrize("tile", [4, 5, 6, 7])
@pytest.mark.parametrize("splits", [1, 3])
def test_small_tiles_fused_epilogue_ragged(tile, splits):
    """The grid-filling tiles with bias + GELU (+ aux) and split-K on a ragged GPT-2-like shape."""
    M, N, K = 2032, 776, 1536
    torch.manual_seed(4)
    a, b, ref = _operands(M, N, K, False, False, torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = _C().gemm(a, b, bias=bias, act=2, aux=aux, tile=tile, splits=splits)
    z = ref + bias
    torch.testing.assert_close(aux.float(), z, rtol=2e-2, atol=2e-2 * K ** 0.5)
    torch.testing.assert_close(y.float(), torch.nn.functional.gelu(aux.float()), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("tile", [8, 9, 10, 11, 12])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("shape,splits", [((1536, 1280, 2048), 1), ((1000, 776, 3072), 3), ((6304, 768, 768), 2)])
def test_pingpong_tiles_ragged_split_k(tile, layout, shape, splits):
    """gemm_pp_k on transformer-like shapes: ragged M / N (the last tile shifted back), K split into
    slices that are whole ping-pong steps (64 deep for KS = 2), every operand layout."""
    M, N, K = shape
    a_tr, b_tr = layout[0] == "t", layout[1] == "n"
    if a_tr and M % 8:
        M += 8 - M % 8
    if b_tr and N % 8:
        N += 8 - N % 8
    torch.manual_seed(7)
    a, b, ref = _operands(M, N, K, a_tr, b_tr, torch.bfloat16)
    c = _C().gemm(a, b, a_tr=a_tr, b_tr=b_tr, out_dtype=torch.float32, tile=tile, splits=splits)
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)


@pytest.mark.parametrize("tile", [8, 9, 10, 11, 12])
def test_pingpong_fused_epilogue_bf16(tile):
    M, N, K = 2048, 1024, 768
    torch.manual_seed(3)
    x, w, ref = _operands(M, N, K, False, False, torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    res = _rand(M, N)
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = _C().gemm(x, w, bias=bias, act=2, aux=aux, residual=res, tile=tile, splits=1)
    z = (ref + bias).bfloat16().float()
    want = (F.gelu(z).bfloat16().float() + res.float())
    torch.testing.assert_close(aux.float(), z, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y.float(), want, rtol=2e-2, atol=3e-2)
