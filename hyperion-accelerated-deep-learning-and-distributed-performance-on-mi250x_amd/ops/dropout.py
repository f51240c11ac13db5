"""Graph-safe dropout on the gfx950 counter-based kernel (``csrc/kernels/dropout.hip``).

Reference: ``nn.Dropout`` (p = 0.1) in every ``nn.TransformerEncoderLayer`` of the LM / custom
Transformer configs and PEFT's LoRA dropout (p = 0.05) — torch's philox ``fused_dropout`` with a
stored bool mask, plus ``masked_scale`` in backward (SURVEY §2.4 "Dropout").

Here the keep mask is never stored: forward and backward regenerate it from the same (seed,
offset) record drawn from torch's default generator (``_native.rng_state``), so a step captured
in a hipGraph draws a fresh mask on every replay and the backward costs one pass over dy.
``Dropout`` is a drop-in ``nn.Dropout`` (no parameters, same repr / state dict).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


def _native_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and _native.use_native(x, op="dropout"))


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        st = _native.rng_state(x.device)
        ctx.st, ctx.p = st, p
        _native.count("dropout")
        return _native.native().dropout(x, p, st)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        return _native.native().dropout(dy, ctx.p, ctx.st), None


def dropout(x: torch.Tensor, p: float = 0.5, training: bool = True) -> torch.Tensor:
    """``F.dropout`` with a regenerated (never stored), graph-safe mask on gfx950."""
    if not training or p == 0.0:
        return x
    if _native_ok(x) and 0.0 < p < 1.0:
        return _native.apply_fn(_DropoutFn, x, float(p))
    return F.dropout(x, p, training)


def keep_mask(x: torch.Tensor, p: float, state: torch.Tensor) -> torch.Tensor:
    """The scaled keep mask keep/(1-p) of ``dropout(x)`` drawn with ``state`` (shape / dtype of x)."""
    return _native.native().dropout(x, p, state, mask=True)


class Dropout(nn.Dropout):
    """``nn.Dropout`` on the graph-safe native kernel."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if self.inplace:
            return F.dropout(x, self.p, self.training, inplace=True)
        return dropout(x, self.p, self.training)
