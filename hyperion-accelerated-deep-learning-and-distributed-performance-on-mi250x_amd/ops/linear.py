"""Linear layers in the weight-streaming regime (a few hundred tokens x large weights).

Reference: the Llama-2-7B LoRA fine-tune (``distributed_utils.py:415-554``, batch 1 x 128 tokens)
runs every projection as ``torch.nn.functional.linear`` → hipBLASLt.  At M = 128 tokens a
4096 x 4096 projection is a 64-workgroup launch that streams its 32 MiB weight at ~0.6 TB/s on
MI355X (profiles/llama_r01).  ``linear_nt`` / ``linear_nn`` (``csrc/kernels/conv_igemm.hip`` with
R = S = 1) split the reduction until ~320 workgroups stream disjoint weight slices with a
multi-stage global_load_lds ring, and the data gradient reads the SAME row-major weight
transposed in-kernel (ds_read_b64_tr_b16) — no ``w.t().contiguous()`` copy.

``linear(x, w, b)``: native forward when M <= ``SKINNY_MAX_M`` tokens and the shapes fit the
kernel (in % 64, out % 8); native data gradient when out % 64 and in % 8; otherwise the vendor
GEMM.  Above ``SKINNY_MAX_M`` tokens the three GEMMs go to the deep-pipelined tiled MFMA kernel
(``ops.gemm``: bias fused in the forward epilogue, W read transposed in the data gradient, no
copies) wherever it is at least as fast as the vendor GEMM for that shape.  The bias gradient is
``csrc/kernels/reduce.hip``'s column sum at any size; the weight gradient (only for trainable
weights) is the split-K MFMA weight-gradient kernel when its output is small (``linear_wgrad``),
else the tiled kernel (or the vendor GEMM).
"""
from __future__ import annotations

import os
import weakref
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native
from . import linear_f32 as _lf32
from .gemm import mm_nn, mm_nt, mm_tn

SKINNY_MAX_M = int(os.environ.get("HYPERION_SKINNY_MAX_M", "1024"))


def _fwd_ok(x2: torch.Tensor, w: torch.Tensor) -> bool:
    return (x2.dtype in (torch.bfloat16, torch.float16) and w.dtype == x2.dtype and x2.shape[0] <= SKINNY_MAX_M
            and x2.shape[1] % 64 == 0 and w.shape[0] % 8 == 0 and w.is_contiguous()
            and _native.use_native(x2, w, op="linear"))


def _bwd_ok(dy2: torch.Tensor, w: torch.Tensor) -> bool:
    return (dy2.dtype == w.dtype and dy2.dtype in (torch.bfloat16, torch.float16) and dy2.shape[0] <= SKINNY_MAX_M
            and w.shape[0] % 64 == 0 and w.shape[1] % 8 == 0 and w.is_contiguous()
            and _native.use_native(dy2, w, op="linear"))


def linear_fwd(x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``x2 @ w.T`` for 2D ``x2`` (native when the shape fits, else the vendor GEMM)."""
    if x2.is_cuda and _fwd_ok(x2, w):
        return _native.native().linear_nt(x2.contiguous(), w)
    y = mm_nt(x2, w) if x2.is_cuda else None
    return y if y is not None else F.linear(x2, w)


def linear_dgrad(dy2: torch.Tensor, w: torch.Tensor, addend: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``dy2 @ w`` (the data gradient of ``linear_fwd``) ``+ addend`` (2D, in the GEMM epilogue —
    a residual branch's gradient of the same input; ``ResidualLink``)."""
    if dy2.is_cuda and _bwd_ok(dy2, w):
        dx = _native.native().linear_nn(dy2.contiguous(), w)
        return dx if addend is None else dx + addend
    if addend is not None:
        addend = addend.to(dy2.dtype)
    dx = mm_nn(dy2, w, residual=addend) if dy2.is_cuda else None
    if dx is not None:
        return dx
    return dy2 @ w if addend is None else torch.addmm(addend, dy2, w)


def arm_link(link, x: torch.Tensor):
    """``link`` (an ``ops.conv.ResidualLink`` on a residual-block input) if ``x`` is its source: the
    op consuming x will add the residual branch's parked gradient into its data gradient."""
    if link is not None and x is link.src and torch.is_grad_enabled():
        link.armed = True
        return link
    return None


def take_link_grad(link, shape) -> Optional[torch.Tensor]:
    """The parked residual gradient for this op's data gradient (2D), consumed."""
    if link is None or link.dres is None:
        return None
    d, link.dres = link.dres, None
    _native.count("residual_grad_fused")
    return d.reshape(-1, shape[-1])


# Weight gradients whose output is small (out x in <= WGRAD_NATIVE_MAX elements) run on the
# split-K MFMA weight-gradient kernel (conv_wgrad.hip at 1x1): at these shapes it beats the vendor
# TN GEMM, which under-fills the chip (MI355X, scripts/gemm_shapes.py: [6304x768]ᵀ[6304x768]
# 28.7 vs 48.4 us; LM-256 FFN [4064x2048]ᵀ[4064x256] 22 vs 32 us; [4064x256]ᵀ[4064x2048] 19.7 vs
# 32.8 us) and loses on larger ones (6304 x 768 -> 3072: 94 vs 68 us).
WGRAD_NATIVE_MAX = int(os.environ.get("HYPERION_WGRAD_NATIVE_MAX", str(1 << 18)))


def linear_wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """``dy2ᵀ @ x2`` (the weight gradient of ``linear_fwd``) in the operands' dtype."""
    M, N = dy2.shape
    K = x2.shape[1]
    if (dy2.is_cuda and dy2.dtype == x2.dtype and dy2.dtype in (torch.bfloat16, torch.float16)
            and N * K <= WGRAD_NATIVE_MAX and K % 64 == 0 and N % 8 == 0 and M < (1 << 22)
            and dy2.is_contiguous() and x2.is_contiguous() and _native.use_native(dy2, op="wgrad")):
        _native.count("linear_wgrad")
        return _native.native().conv_wgrad(dy2.view(M, N, 1, 1), x2.view(M, K, 1, 1), 1, 1, 1, 1, 0, 0).view(N, K)
    dw = mm_tn(dy2, x2) if dy2.is_cuda else None
    return dw if dw is not None else dy2.t() @ x2


def bias_grad(dy2: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """``dy2.sum(0)`` (a bias gradient) — ``csrc/kernels/reduce.hip`` column sums on gfx950 (autograd's
    generic reduction ran [6304, 768] bf16 at 0.4 TB/s in the ViT step)."""
    if (dy2.is_cuda and dy2.dtype in (torch.bfloat16, torch.float16, torch.float32) and dy2.shape[-1] % 8 == 0
            and dy2.is_contiguous() and dy2.data_ptr() % 16 == 0 and dy2.numel() > 0
            and _native.use_native(dy2, op="bias_grad")):
        return _native.native().column_sum(dy2, dtype)
    return dy2.sum(0, dtype=torch.float32).to(dtype)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, link=None, blink=None):
        x2 = x.reshape(-1, x.shape[-1])
        y = None
        if b is not None and not _fwd_ok(x2, w):
            y = mm_nt(x2, w, bias=b) if x2.is_cuda else None  # bias in the tiled kernel's epilogue
            if y is None:
                y = F.linear(x2, w, b.to(x2.dtype))  # ... or the vendor GEMM's
        else:
            y = linear_fwd(x2, w)
            if b is not None:
                y = y + b.to(y.dtype)
        ctx.save_for_backward(x2 if ctx.needs_input_grad[1] else None, w)
        ctx.has_b = b is not None
        ctx.bdt = b.dtype if b is not None else None
        ctx.xshape = x.shape
        ctx.link = link
        ctx.blink = blink
        if blink is not None and b is not None:
            blink.armed = True  # the consuming norm's backward will sum our output's gradient
            blink.dtype = b.dtype
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(w.dtype)
        add = take_link_grad(ctx.link, ctx.xshape)
        dx = linear_dgrad(dy2, w, add).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = linear_wgrad(dy2.contiguous(), x2.contiguous()).to(w.dtype) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = ctx.blink.take(dy) if ctx.blink is not None else None
            if db is not None:
                _native.count("bias_grad_from_norm")
                db = db.to(ctx.bdt)
            else:
                db = bias_grad(dy2.contiguous(), ctx.bdt)
        elif ctx.blink is not None:
            ctx.blink.take(dy)
        return dx, dw, db, None, None


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None, link=None,
           blink=None) -> torch.Tensor:
    """``F.linear`` with the weight-streaming kernels on gfx950 (same math, same grads).  Under
    autocast, x and w are cast to the autocast dtype first (differentiable casts, like torch's own
    autocast of ``F.linear``), so the native kernels serve the AMP trainers too.  ``link``: a
    ``ResidualLink`` on x (see :func:`arm_link`)."""
    if not (x.is_cuda and _native.use_native(x, op="linear")) or _native.plain_fp32(x):
        if _native.plain_fp32(x) and _lf32.applies(x, w):
            return _lf32.linear_f32(x, w, b)  # large fp32 GEMMs: native fp32 MFMA where it is faster
        return F.linear(x, w, b)
    if torch.is_autocast_enabled(x.device.type):
        dt = torch.get_autocast_dtype(x.device.type)
        if dt not in (torch.bfloat16, torch.float16):
            return F.linear(x, w, b)
        with torch.autocast(x.device.type, enabled=False):
            return _native.apply_fn(_LinearFn, x.to(dt), w.to(dt), b)  # (a cast copy: the link stays unarmed)
    link = arm_link(link, x)
    y = _native.apply_fn(_LinearFn, x, w, b, link, blink)
    if link is not None and y.grad_fn is not None:
        link.first_node = weakref.ref(y.grad_fn)
    return y


class Linear(nn.Linear):
    """``nn.Linear`` (same parameters and state-dict keys) routed through :func:`linear`."""

    def forward(self, x: torch.Tensor, link=None, blink=None) -> torch.Tensor:  # type: ignore[override]
        return linear(x, self.weight, self.bias, link=link, blink=blink)
