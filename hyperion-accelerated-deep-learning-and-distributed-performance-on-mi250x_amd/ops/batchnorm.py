"""Fused BatchNorm (+ residual add) (+ ReLU) — the conv epilogue of every ResNet block.

Reference: torchvision ResNet blocks run ``conv -> bn -> relu`` and ``bn3 -> += identity ->
relu`` as three or four separate kernels (MIOpen BN, elementwise add, ReLU) per block
(``baseline_performance.ipynb:203-205``; SURVEY §2.4 "Convolution + BatchNorm + ReLU").

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` subclass (same parameters, buffers and
state-dict keys) whose forward takes an optional ``residual`` and applies ReLU when
``act=True``.  On GPU with channels-last activations it runs the gfx950 kernels in
``csrc/kernels/bn_act.hip``: one stats pass (atomic per-channel sums) + one apply pass forward
that finalizes inline (residual + ReLU folded into the apply), one reduce pass + one dx pass
backward (ReLU mask from the saved output, residual gradient written by the same pass).  Elsewhere it runs the PyTorch reference composition, which
is also the test oracle.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


def bn_act_reference(
    x: torch.Tensor,
    residual: Optional[torch.Tensor],
    weight: Optional[torch.Tensor],
    bias: Optional[torch.Tensor],
    running_mean: Optional[torch.Tensor],
    running_var: Optional[torch.Tensor],
    training: bool,
    momentum: float,
    eps: float,
    act: bool,
) -> torch.Tensor:
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    if act:
        y = F.relu(y)
    return y


def _native_ok(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dtype not in _native.DTYPE_CODE:
        return False
    if x.dim() == 4:
        if not x.is_contiguous(memory_format=torch.channels_last):
            return False
    elif x.dim() != 2 or not x.is_contiguous():
        return False
    C = x.shape[1]
    if C % 8:
        return False
    cv = C // 8
    return cv <= 256 or cv % 256 == 0


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, momentum, eps, training, act):
        C = _native.native()
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        if residual is not None and x.dim() == 4 and not residual.is_contiguous(memory_format=torch.channels_last):
            residual = residual.contiguous(memory_format=torch.channels_last)
        sums = _native.zeroed(_native.STAT_SLOTS * 2 * x.shape[1], x.device) if training else None
        ctx.bsums = _native.zeroed(_native.STAT_SLOTS * 2 * x.shape[1], x.device)  # the backward's Σdz, Σdz·x (same fill)
        y, mean, invstd = C.bn_fwd(x, residual, weight, bias, running_mean, running_var, momentum, eps, training, act,
                                   sums=sums)
        ctx.act = act
        ctx.training = training
        ctx.has_res = residual is not None
        # training without a residual: the backward recomputes the ReLU mask from x (one stream
        # fewer to read); otherwise it needs the forward output
        keep_y = act and (residual is not None or not training)
        ctx.save_for_backward(x, y if keep_y else None, weight, bias, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, bias, mean, invstd = ctx.saved_tensors
        need_res = ctx.has_res and ctx.needs_input_grad[1]
        bsums, ctx.bsums = ctx.bsums, None  # a second backward (retain_graph) takes fresh zeros
        dx, dres, dw, db = _native.native().bn_bwd(
            dy, x, y, weight, bias, mean, invstd, ctx.training, ctx.act, need_res, sums=bsums
        )
        return (
            dx if ctx.needs_input_grad[0] else None,
            dres if need_res else None,
            dw if (weight is not None and ctx.needs_input_grad[2]) else None,
            db if ctx.needs_input_grad[3] else None,
            None, None, None, None, None, None,
        )


def bn_act(
    x: torch.Tensor,
    residual: Optional[torch.Tensor],
    weight: Optional[torch.Tensor],
    bias: Optional[torch.Tensor],
    running_mean: Optional[torch.Tensor],
    running_var: Optional[torch.Tensor],
    training: bool,
    momentum: float,
    eps: float,
    act: bool,
) -> torch.Tensor:
    """Functional fused BN(+res)(+ReLU); dispatches to HIP when possible."""
    if (
        _native.use_native(x, op="bn")
        and _native_ok(x)
        and (weight is None or weight.dtype == torch.float32)
        and (running_mean is None or running_mean.dtype == torch.float32)
    ):
        return _native.apply_fn(_BNActFn, x, residual, weight, bias, running_mean, running_var, momentum, eps, training, act)
    return bn_act_reference(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, act)


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` + optional residual add + optional ReLU, fused on gfx950."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: Optional[float] = 0.1, act: bool = False,
                 **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        self.act = act
        self._host_batches = 0  # mirrors num_batches_tracked without a per-step device launch

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={self.act}"

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        if self.track_running_stats and self.num_batches_tracked is not None and self._host_batches:
            with torch.no_grad():
                self.num_batches_tracked.add_(self._host_batches)
            self._host_batches = 0
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        # the loaded num_batches_tracked is the whole count: drop any un-flushed host increments
        self._host_batches = 0
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:  # type: ignore[override]
        use_batch_stats = self.training or not self.track_running_stats
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats:
            if self.momentum is None:  # cumulative moving average needs the true count every step
                self.num_batches_tracked.add_(1)
                momentum = 1.0 / float(self.num_batches_tracked.item())
            else:
                self._host_batches += 1
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        return bn_act(x, residual, self.weight, self.bias, rm, rv, use_batch_stats, momentum, self.eps, self.act)


class HostCounterReplay:
    """Keeps ``BatchNormAct2d``'s host-side ``num_batches_tracked`` mirror right under hipGraph
    replay: a captured step increments the mirror once in Python while recording (a forward that
    never ran on the device) and never again, so ``TrainStep`` / ``GraphedClosure`` snapshot the
    mirrors around the capture, undo the recording pass, and add the per-step delta on every
    replay — checkpoints then store the true count, like torch's BatchNorm."""

    def __init__(self, module: nn.Module):
        self.mods = [m for m in module.modules() if hasattr(m, "_host_batches")]
        self.before = [m._host_batches for m in self.mods]
        self.delta: list = []

    def captured(self) -> "HostCounterReplay":
        self.delta = [(m, m._host_batches - b) for m, b in zip(self.mods, self.before) if m._host_batches != b]
        for m, d in self.delta:
            m._host_batches -= d
        return self

    def replayed(self, n: int = 1) -> None:
        for m, d in self.delta:
            m._host_batches += n * d


class BatchNormAct1d(BatchNormAct2d):
    """[N, C] variant (same kernels; rows = batch)."""

    def _check_input_dim(self, input):
        if input.dim() != 2:
            raise ValueError(f"expected 2D input (got {input.dim()}D input)")
