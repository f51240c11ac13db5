"""Global-norm clipping keeps one pointer table per model: two same-shaped models in
one process never clip each other's gradients, and many models can be clipped (regression: a
WeakKeyDictionary keyed by tensors raised on hash-bucket collisions)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_clip_tables_per_model_and_many_models():
    from hyperion.ops.optim import clip_grad_norm_

    models = [torch.nn.Linear(64, 64).cuda() for _ in range(64)]
    for i, m in enumerate(models):
        for p in m.parameters():
            p.grad = torch.full_like(p, float(i + 1))
    norms = [clip_grad_norm_(list(m.parameters()), 1e9) for m in models]
    for i, (m, n) in enumerate(zip(models, norms)):
        ref = torch.cat([torch.full((p.numel(),), float(i + 1)) for p in m.parameters()]).norm()
        assert abs(float(n) - float(ref)) <= 1e-3 * float(ref)
    # clip one model; the other's gradients are untouched
    clip_grad_norm_(list(models[0].parameters()), 0.5)
    assert float(models[1].weight.grad[0, 0]) == 2.0
    assert float(torch.cat([p.grad.flatten() for p in models[0].parameters()]).norm()) <= 0.5 + 1e-4
