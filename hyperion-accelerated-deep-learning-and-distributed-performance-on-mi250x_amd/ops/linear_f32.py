"""fp32 linear layers on the fp32-input MFMA GEMM (``csrc/kernels/gemm_f32.hip``).

Reference: the fp32 rows of the reference-methodology benchmarks run every ``nn.Linear`` /
``nn.TransformerEncoderLayer`` GEMM on hipBLASLt in fp32 (``Phase 1/baseline_performance.ipynb:
252-358`` ViT-B/16 / CustomTransformer; ``02_development/compilation_optimization.py:47-51``;
SURVEY §2.4 "GEMM").  Here the three GEMMs of an fp32 linear layer — forward ``x Wᵀ (+ b)``, data
gradient ``dy W`` (W read transposed in-kernel) and weight gradient ``dyᵀ x`` (both operands read
transposed) — can run on the native fp32 kernel with no transposed copies.

Routing ("measure, don't guess"): per GEMM shape the first eager call times the vendor GEMM and the
native kernel at its tuned launch plan (``conv_f32.gemm``) and keeps the faster; a capture takes the
cached choice (vendor for a shape never seen eagerly).  Layers below ``MIN_MACS`` multiply-adds per
GEMM stay plain ``F.linear``: an autograd Function costs ~20-30 us of host time per layer, which a
launch-bound fp32 model (the 512-token CustomTransformer) cannot hide (``ops/_native.py``
``plain_fp32``).  ``HYPERION_LINEAR_F32=0`` disables the path.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from . import _native
from . import conv_f32

ENABLED = os.environ.get("HYPERION_LINEAR_F32", "1") == "1"
MIN_MACS = int(os.environ.get("HYPERION_LINEAR_F32_MIN_MACS", str(1 << 31)))
_CHOICE: Dict[Tuple, bool] = {}  # (op, M, N, K) -> native faster


def applies(x: torch.Tensor, w: torch.Tensor) -> bool:
    if not (ENABLED and x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() >= 2):
        return False
    tokens = x.numel() // x.shape[-1]
    return (tokens * w.shape[0] * w.shape[1] >= MIN_MACS and w.shape[1] % 4 == 0 and w.shape[0] % 4 == 0
            and w.is_contiguous() and _native.use_native(x, op="linear"))


def _choose(key: Tuple, native: Callable[[], torch.Tensor], vendor: Callable[[], torch.Tensor]) -> torch.Tensor:
    c = _CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return vendor()
        from .gemm import _time

        native()  # tunes the native launch plan for the shape
        c = _time(native, reps=3) < _time(vendor, reps=3)
        _CHOICE[key] = c
    if c:
        _native.count("linear_f32")
        return native()
    return vendor()


class _LinearF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        M, K, N = x2.shape[0], x2.shape[1], w.shape[0]
        y = _choose(("fwd", M, N, K, b is not None), lambda: conv_f32.gemm(x2, w, bias=b),
                    lambda: F.linear(x2, w, b))
        ctx.save_for_backward(x2, w)
        ctx.has_b = b is not None
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        N = w.shape[0]
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        M, K = x2.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _choose(("dgrad", M, K, N), lambda: conv_f32.gemm(dy2, w, b_tr=True), lambda: dy2 @ w)
            dx = dx.view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = _choose(("wgrad", N, K, M), lambda: conv_f32.gemm(dy2, x2, a_tr=True, b_tr=True), lambda: dy2.t() @ x2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dx, dw, db


def linear_f32(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    return _native.apply_fn(_LinearF32Fn, x, w, b)
