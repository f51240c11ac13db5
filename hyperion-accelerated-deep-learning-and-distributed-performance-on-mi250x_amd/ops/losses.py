"""Fused losses.

Reference: the step benchmark's ``nn.MSELoss()`` against random ``(32, 1000)`` targets
(``Phase 1/baseline_performance.ipynb:252-358``) — on bf16 logits torch runs a cast to fp32, the
difference, the square and a mean forward, and three elementwise kernels backward.  ``mse_loss``
computes the fp32 mean and the gradient ``2 (x - t) / n`` in ONE native pass (``reduce.hip``);
backward only scales the saved gradient by the incoming scalar.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native

_MAX_FUSED = 1 << 20  # one-block kernel: small outputs (logits), larger tensors take torch's ops


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, t):
        loss, g = _native.native().mse_fwd_bwd(x.contiguous(), t.float().contiguous())
        ctx.save_for_backward(g)
        return loss

    @staticmethod
    def backward(ctx, go):
        (g,) = ctx.saved_tensors
        return g * go, None  # (a 0-dim fp32 go does not promote g: one kernel, g's dtype)


def mse_loss(x: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """``F.mse_loss(x.float(), target)`` (mean reduction), fused on gfx950 for small tensors."""
    if (x.is_cuda and x.shape == target.shape and 0 < x.numel() <= _MAX_FUSED and not target.requires_grad
            and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and _native.use_native(x, op="mse")):
        _native.count("mse_fused")
        return _MSEFn.apply(x, target)
    return F.mse_loss(x.float(), target.float())


class MSELoss(nn.MSELoss):
    """``nn.MSELoss()`` (mean) computed by :func:`mse_loss`; takes low-precision inputs directly
    (``accepts_low_precision``: the training step skips its fp32 cast of the logits)."""

    accepts_low_precision = True

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if self.reduction != "mean":
            return super().forward(input.float(), target)
        return mse_loss(input, target)
