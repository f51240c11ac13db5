"""One-launch column sums (reduce.hip colsum_last_block, opt-in ``colsum_set_fused``): the
last-arriving block of each column slab combines the partial rows — bias gradients without the
second (combine) launch (measured slower than two launches on MI355X: the per-block agent-scope
release is an L2 write-back; kept as a tested option).  Checked against
torch's fp32 sums, run-to-run bit-exact (fixed combine order), under graph replay (the ticket
slots reset themselves) and in the activation-backward + bias-gradient kernel."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused():
    from hyperion.ops import _native

    C = _native.native()
    C.colsum_set_fused(64)
    yield C
    C.colsum_set_fused(0)  # the default: two launches (measured faster)


@pytest.mark.parametrize("shape", [(8192, 768), (6304, 3072), (17, 64), (3, 4096), (1000, 520), (65536, 8)])
@pytest.mark.parametrize("dt,odt", [(torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
                                    (torch.float32, torch.float32)])
def test_column_sum_one_launch_matches_fp32(_fused, shape, dt, odt):
    C = _fused
    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dt)
    ref = x.float().sum(0)
    a = C.column_sum(x, odt)
    b = C.column_sum(x, odt)
    torch.cuda.synchronize()
    assert torch.equal(a, b)  # deterministic combine order
    torch.testing.assert_close(a.float(), ref.to(odt).float(), rtol=1e-2 if odt != torch.float32 else 1e-4,
                               atol=1e-2 if odt != torch.float32 else 1e-3)
    C.colsum_set_fused(0)
    c = C.column_sum(x, odt)  # the two-launch path
    torch.testing.assert_close(a.float(), c.float(), rtol=1e-2, atol=1e-2)


def test_column_sum_one_launch_graph_replay(_fused):
    C = _fused
    x = torch.randn(4096, 1024, device="cuda").bfloat16()
    out = [None]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            out[0] = C.column_sum(x, torch.float32)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out[0] = C.column_sum(x, torch.float32)
        out.append(C.column_sum(x * 2, torch.float32))
    ref = x.float().sum(0)
    for i in range(3):
        x.copy_(torch.randn_like(x.float()).bfloat16())
        ref = x.float().sum(0)
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out[0], ref, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(out[1], 2 * ref, rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("act", [1, 2])
def test_act_bwd_colsum_one_launch(_fused, act):
    C = _fused
    torch.manual_seed(1)
    dh = torch.randn(6304, 3072, device="cuda").bfloat16()
    z = torch.randn(6304, 3072, device="cuda").bfloat16()
    dy, db = C.act_bwd_colsum(dh, z, act, torch.float32, 0.0, None)
    C.colsum_set_fused(0)
    dy2, db2 = C.act_bwd_colsum(dh, z, act, torch.float32, 0.0, None)
    torch.cuda.synchronize()
    assert torch.equal(dy, dy2)
    torch.testing.assert_close(db, dy.float().sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(db, db2, rtol=1e-5, atol=1e-3)
