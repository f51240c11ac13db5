"""Update-level parity checks for captured-vs-eager training steps.

Comparing parameters after a few Adam steps with an absolute tolerance cannot fail: the whole
update is ~lr per element per step, so a captured step that applied half an update, skipped the
optimizer once or reused a stale gradient lands inside ``atol=2e-3`` too.  These helpers compare
what the steps DID instead:

* :func:`update_rel_err` — ‖Δ_a − Δ_b‖ / ‖Δ_b‖ over all parameters, Δ = after − before from the
  SAME starting point (a skipped step or a stale gradient moves this by O(1/steps));
* :func:`assert_losses_match` — the per-step losses, which see every forward the schedule ran.

``tests/test_parity_cpu.py`` shows on CPU that both checks fail on deliberately broken schedules.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Optional

import torch


def snapshot(named: Iterable) -> Dict[str, torch.Tensor]:
    """fp64 CPU copies of ``(name, tensor)`` pairs (a ``named_parameters()`` or state-dict items)."""
    return {k: v.detach().to(torch.float64).cpu().clone() for k, v in named}


def update_rel_err(before: Dict[str, torch.Tensor], after_a: Dict[str, torch.Tensor],
                   after_b: Dict[str, torch.Tensor], keys: Optional[Iterable[str]] = None) -> float:
    """‖Δ_a − Δ_b‖₂ / ‖Δ_b‖₂ with Δ_x = after_x − before, summed over ``keys`` (default: all of
    ``before``).  ``after_b`` is the reference schedule (eager)."""
    num = 0.0
    den = 0.0
    for k in (keys if keys is not None else before.keys()):
        b0 = before[k].to(torch.float64)
        da = after_a[k].detach().to(torch.float64).cpu() - b0
        db = after_b[k].detach().to(torch.float64).cpu() - b0
        num += float((da - db).pow(2).sum())
        den += float(db.pow(2).sum())
    assert den > 0, "the reference schedule did not move any parameter"
    return math.sqrt(num / den)


def assert_update_parity(before, after_a, after_b, rel: float = 2e-2, keys=None, what: str = "") -> float:
    err = update_rel_err(before, after_a, after_b, keys)
    assert err < rel, f"{what} update mismatch: ||d_a - d_b|| / ||d_b|| = {err:.3e} >= {rel:.1e}"
    return err


def assert_losses_match(losses_a, losses_b, rtol: float = 5e-3, atol: float = 1e-5, what: str = "") -> None:
    la = torch.tensor([float(v) for v in losses_a], dtype=torch.float64)
    lb = torch.tensor([float(v) for v in losses_b], dtype=torch.float64)
    assert la.shape == lb.shape, f"{what} step counts differ: {la.numel()} vs {lb.numel()}"
    torch.testing.assert_close(la, lb, rtol=rtol, atol=atol, msg=lambda m: f"{what} per-step losses differ: {m}")
