"""Dropout masks across SPLIT hipGraphs: forward captured in graph 1, backward in
graph 2 (TrainStep's split-backward schedule).  Every replay rewrites the generator's extragraph
offset, so the backward must read the snapshot its forward's graph took (csrc/bindings/rng_ops.cpp),
not the live offset — otherwise it regenerates a different mask."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_dropout_mask_matches_across_graphs():
    from hyperion.ops import _native
    from hyperion.ops.dropout import dropout

    assert _native.available()
    x = torch.ones(1 << 16, device="cuda", requires_grad=True)
    dy = torch.ones(1 << 16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up
        for _ in range(2):
            y = dropout(x, 0.5)
            torch.autograd.grad(y, x, dy)
    torch.cuda.current_stream().wait_stream(s)
    _native.reset_counters()
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        y = dropout(x, 0.5)
    with torch.cuda.graph(g2, pool=g1.pool()):
        (gx,) = torch.autograd.grad(y, x, dy)
    assert _native.counters().get("dropout", 0) == 1  # the native kernel was captured
    seen = []
    for _ in range(3):
        g1.replay()
        g2.replay()
        torch.cuda.synchronize()
        # x = dy = 1: forward output and input gradient are both keep / (1 - p)
        assert torch.equal(gx, y), "backward regenerated a different mask than its forward"
        frac = float((y == 0).float().mean())
        assert 0.45 < frac < 0.55
        seen.append(y.clone())
    assert not torch.equal(seen[0], seen[1])  # a fresh mask per replay
