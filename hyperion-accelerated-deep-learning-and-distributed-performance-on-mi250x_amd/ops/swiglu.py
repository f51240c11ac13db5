"""SwiGLU ``silu(gate) * up`` as one gfx950 kernel (fwd and bwd).

Reference: HF ``LlamaMLP`` (``down_proj(act_fn(gate_proj(x)) * up_proj(x))``) inside the Llama
fine-tune (C26) — silu and mul are separate kernels there, with silu's output kept for backward.
Here the forward writes only ``h``; backward recomputes the sigmoid from ``gate``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, u):
        ctx.save_for_backward(g, u)
        return _native.native().swiglu_fwd(g, u)

    @staticmethod
    def backward(ctx, dh):
        g, u = ctx.saved_tensors
        dg, du = _native.native().swiglu_bwd(dh.contiguous(), g, u)
        return dg, du


def swiglu(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    if (_native.use_native(gate, up, op="swiglu") and gate.dtype in _native.DTYPE_CODE and gate.dtype == up.dtype
            and gate.shape == up.shape and gate.numel() % 8 == 0):
        return _native.apply_fn(_SwiGLUFn, gate, up)
    return F.silu(gate) * up
