"""Deferred global-norm clip (clip_grad_norm_(defer_to=FusedAdam)): the coefficient applied inside
the Adam step equals clipping the gradients first (CPU reference path; the GPU kernel takes the same
coefficient through its inv_scale operand)."""
import torch

from hyperion.ops.optim import FusedAdam, clip_grad_norm_


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _grads(m):
    torch.manual_seed(1)
    x = torch.randn(8, 16)
    (m(x).pow(2).sum() * 50.0).backward()  # large grads: the clip is active


def test_deferred_clip_matches_eager_clip():
    a, b = _model(0), _model(0)
    oa = FusedAdam(a.parameters(), lr=1e-2, weight_decay=0.01, adamw=True)
    ob = FusedAdam(b.parameters(), lr=1e-2, weight_decay=0.01, adamw=True)
    for _ in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            _grads(m)
        na = clip_grad_norm_(a.parameters(), 1.0)
        nb = clip_grad_norm_(b.parameters(), 1.0, defer_to=ob)
        assert float(na) > 1.0 and torch.allclose(na, nb)
        assert ob.clip_coef is not None
        oa.step()
        ob.step()
        assert ob.clip_coef is None  # consumed by the step
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, atol=1e-6, rtol=1e-5)
