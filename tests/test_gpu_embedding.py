"""Token embedding gather + deterministic sorted-run backward vs nn.functional.embedding."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("V,E,shape,pad", [(50257, 256, (32, 127), None), (32000, 4096, (1, 128), 0),
                                           (100, 64, (7, 33), 3)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_fwd_bwd_match(V, E, shape, pad, dtype):
    from hyperion.ops.embedding import embedding

    torch.manual_seed(0)
    w = torch.randn(V, E, device="cuda").to(dtype).requires_grad_(True)
    ids = torch.randint(0, min(V, 500), shape, device="cuda")  # many repeats
    y = embedding(ids, w, pad)
    g = torch.randn_like(y)
    y.backward(g)
    wr = w.detach().float().requires_grad_(True)
    yr = F.embedding(ids, wr, pad)
    yr.backward(g.float())
    torch.testing.assert_close(y.float(), yr)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=2e-2, atol=2e-2)
    w.grad = None
    embedding(ids, w, pad).backward(g)
    g1 = w.grad.clone()
    w.grad = None
    embedding(ids, w, pad).backward(g)
    assert (g1.float() - w.grad.float()).abs().max() <= 1e-2 * g1.float().abs().max() + 1e-3
