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


class _LinearMSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, t):
        loss, dz = _native.native().linear_mse_fwd(x, w, b, t)
        ctx.save_for_backward(dz, x, w)
        ctx.with_bias = b is not None
        return loss

    @staticmethod
    def backward(ctx, go):
        dz, x, w = ctx.saved_tensors
        dx, dw, db = _native.native().linear_mse_bwd(dz, go.float().reshape(1), x, w, ctx.with_bias)
        return dx, dw, db, None


def linear_mse(x: torch.Tensor, weight: torch.Tensor, bias, target: torch.Tensor) -> torch.Tensor:
    """``F.mse_loss(F.linear(x, weight, bias).float(), target)`` (mean): the classifier head and the
    loss as two native launches (``linear_mse.hip``: forward + loss, then dX / dW / db in one
    backward launch) instead of the unfused path's 11 small kernels.  Logits are rounded to the
    compute dtype as the unfused head would produce them; everything else accumulates in fp32."""
    M = x.shape[0] if x.dim() == 2 else 0
    if (x.is_cuda and x.dim() == 2 and weight.dim() == 2 and 1 <= M <= 64 and x.shape[1] % 8 == 0
            and x.dtype == weight.dtype and (bias is None or bias.dtype == x.dtype)
            and x.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and target.shape == (M, weight.shape[0]) and not target.requires_grad
            and _native.use_native(x, op="linear_mse")):
        _native.count("linear_mse")
        return _LinearMSEFn.apply(x.contiguous(), weight.contiguous(),
                                  None if bias is None else bias.contiguous(), target.float().contiguous())
    return F.mse_loss(F.linear(x, weight, bias).float(), target.float())


class LinearMSELoss(nn.Module):
    """The classifier ``head`` (an ``nn.Linear``) and ``nn.MSELoss()`` as one loss: ``forward(features,
    target) == MSELoss()(head(features), target)``.  Used with a model whose ``head_in_loss`` is set
    (it then returns the pooled features); the head's parameters stay the model's own, so optimizers,
    DDP buckets and checkpoints see them unchanged."""

    accepts_low_precision = True

    def __init__(self, head: nn.Linear):
        super().__init__()
        self.head = [head]  # not a submodule: the model owns (and registers) the parameters

    def forward(self, features: torch.Tensor, target: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        h = self.head[0]
        return linear_mse(features, h.weight, h.bias, target)


class MSELoss(nn.MSELoss):
    """``nn.MSELoss()`` (mean) computed by :func:`mse_loss`; takes low-precision inputs directly
    (``accepts_low_precision``: the training step skips its fp32 cast of the logits)."""

    accepts_low_precision = True

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if self.reduction != "mean":
            return super().forward(input.float(), target)
        return mse_loss(input, target)
