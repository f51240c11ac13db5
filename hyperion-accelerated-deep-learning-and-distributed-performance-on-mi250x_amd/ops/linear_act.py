"""Linear + bias + activation with the activation in the GEMM epilogue (tiled MFMA kernel / hipBLASLt).

Reference: every ``nn.TransformerEncoderLayer`` FFN runs ``linear1`` then ReLU/GELU as separate
kernels (C14/C15/C5), and the ViT MLP likewise.  ``torch._addmm_activation`` asks hipBLASLt for the
bias+ReLU (or bias+GELU) epilogue, so the activation costs no extra pass over the [tokens, ff]
tensor — but it has no autograd formula.  ``linear_act`` wraps it:

* ReLU: forward = one epilogue GEMM; backward masks with the saved OUTPUT (``h > 0`` ⇔ ``y > 0``),
  so the pre-activation is never stored;
* GELU: backward needs the pre-activation: the tiled MFMA kernel (``ops.gemm``) writes BOTH
  ``z = x Wᵀ + b`` (aux output) and ``gelu(z)`` from one epilogue; on the vendor path the forward
  keeps ``z`` (bias epilogue) and applies GELU and the inner dropout as ONE native pass
  (``dropout.hip`` mode 2);
* large-token GEMMs (forward, ``dy W``, ``dyᵀ x``) run on the tiled MFMA kernel where it beats the
  vendor GEMM for the shape (``ops.gemm`` routing);
* backward: the activation backward and the bias gradient are ONE native pass
  (``act_bwd_colsum``: dy written once, its column sums taken from registers), the weight
  gradient on the MFMA split-K kernel when its output is small (``linear.linear_wgrad``).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _native
from . import linear_f32 as _lf32
from . import recompute as _rc
from .gemm import mm_nn, mm_nt
import weakref

from .linear import arm_link, bias_grad, linear_wgrad, take_link_grad


def _act_bwd(dh: torch.Tensor, z: torch.Tensor, act: str, bdt: torch.dtype, need_b: bool, drop=(0.0, None)):
    """(dy, db): the activation backward and, when needed, the bias gradient — one native pass
    (``reduce.hip`` act_bwd_colsum) on gfx950, else autograd's ops.  ``drop`` = (p, rng record): dh
    is the gradient of dropout(act(z)); the mask is regenerated in the same pass."""
    p, st = drop
    if (z.is_cuda and z.dtype in (torch.bfloat16, torch.float16) and z.shape[-1] % 8 == 0 and z.is_contiguous()
            and _native.use_native(z, op="act_bwd")):
        _native.count("act_bwd_colsum")
        dy, db = _native.native().act_bwd_colsum(dh.contiguous(), z, 1 if act == "relu" else 2, bdt, p, st)
        return dy, (db if need_b else None)
    if p > 0.0:
        dh = _native.native().dropout(dh.contiguous(), p, st)
    if act == "relu":
        dy = torch.ops.aten.threshold_backward(dh, z, 0)
    else:
        dy = torch.ops.aten.gelu_backward(dh, z)
    return dy, (bias_grad(dy, bdt) if need_b else None)


def _dgrad(dy: torch.Tensor, wc: torch.Tensor, add: Optional[torch.Tensor] = None) -> torch.Tensor:
    if add is not None:
        add = add.to(dy.dtype)
    dx = mm_nn(dy, wc, residual=add) if dy.is_cuda else None
    if dx is not None:
        return dx
    return dy @ wc if add is None else torch.addmm(add, dy, wc)


def _cdt(x: torch.Tensor) -> torch.dtype:
    return torch.get_autocast_dtype(x.device.type) if torch.is_autocast_enabled(x.device.type) else x.dtype


def _drop_state(x: torch.Tensor, p: float):
    return (p, _native.rng_state(x.device)) if p > 0.0 else (0.0, None)


class _LinearReLU(torch.autograd.Function):
    """``dropout(relu(x Wᵀ + b))`` (p may be 0): bias + ReLU (+ dropout) in the GEMM epilogue; the
    backward masks with the saved OUTPUT (kept elements: h·scale > 0 ⇔ z > 0; dropped: gradient 0)."""

    @staticmethod
    def forward(ctx, x, w, b, p=0.0, link=None):
        dt = _cdt(x)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).to(dt)
        wc, bc = w.to(dt), b.to(dt)
        drop = _drop_state(x2, p)
        ctx.link = link
        h = mm_nt(x2, wc, bias=b, act="relu", dropout_p=drop[0], rng=drop[1]) if x2.is_cuda else None
        if h is None:
            h = torch._addmm_activation(bc, x2, wc.t(), use_gelu=False)
            if drop[0] > 0.0:
                h = _native.native().dropout(h, drop[0], drop[1])
        ctx.save_for_backward(x2, wc, h)
        ctx.meta = (x.dtype, w.dtype, b.dtype, shape)
        ctx.drop = drop
        return h.view(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dh):
        x2, wc, h = ctx.saved_tensors
        xdt, wdt, bdt, shape = ctx.meta
        dy, db = _act_bwd(dh.reshape(h.shape).to(h.dtype), h, "relu", bdt, ctx.needs_input_grad[2], ctx.drop)
        add = take_link_grad(ctx.link, shape)
        dx = _dgrad(dy, wc, add).view(shape).to(xdt) if ctx.needs_input_grad[0] else None
        dw = linear_wgrad(dy, x2.contiguous()).to(wdt) if ctx.needs_input_grad[1] else None
        return dx, dw, db, None, None


class _LinearGELU(torch.autograd.Function):
    """``gelu(x Wᵀ + b)``: bias in the GEMM epilogue, the pre-activation kept for backward."""

    @staticmethod
    def forward(ctx, x, w, b, p=0.0, link=None):
        dt = _cdt(x)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).to(dt)
        wc, bc = w.to(dt), b.to(dt)
        drop = _drop_state(x2, p)
        ctx.link = link
        y = torch.empty(x2.shape[0], w.shape[0], device=x2.device, dtype=dt) if x2.is_cuda else None
        h = mm_nt(x2, wc, bias=b, act="gelu", aux=y, dropout_p=drop[0], rng=drop[1]) if x2.is_cuda else None
        if h is None:
            y = torch.addmm(bc, x2, wc.t())
            if y.is_cuda and y.dtype in (torch.bfloat16, torch.float16) and _native.use_native(y, op="act_dropout"):
                h = _native.native().dropout(y, drop[0], drop[1], act=2)  # GELU + dropout: one pass
            else:
                h = F.gelu(y)
                if drop[0] > 0.0:
                    h = _native.native().dropout(h, drop[0], drop[1])
        ctx.save_for_backward(x2, wc, y)
        ctx.meta = (x.dtype, w.dtype, b.dtype, shape)
        ctx.drop = drop
        if _rc.active() and y.is_cuda and y.dtype in (torch.bfloat16, torch.float16):
            # selective recompute: the next GEMM (fc2) saves this recipe instead of h
            _rc.register(h, lambda: _native.native().dropout(y, drop[0], drop[1], act=2))
        return h.view(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dh):
        x2, wc, y = ctx.saved_tensors
        xdt, wdt, bdt, shape = ctx.meta
        dy, db = _act_bwd(dh.reshape(y.shape).to(y.dtype), y, "gelu", bdt, ctx.needs_input_grad[2], ctx.drop)
        add = take_link_grad(ctx.link, shape)
        dx = _dgrad(dy, wc, add).view(shape).to(xdt) if ctx.needs_input_grad[0] else None
        dw = linear_wgrad(dy, x2.contiguous()).to(wdt) if ctx.needs_input_grad[1] else None
        return dx, dw, db, None, None


def linear_act(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], activation: str,
               dropout_p: float = 0.0, link=None) -> torch.Tensor:
    """``dropout(act(x Wᵀ + b))`` — pass ``dropout_p`` only in training (applied whenever > 0).
    ``link``: a ``ResidualLink`` on x (its parked residual gradient rides the data-gradient GEMM)."""
    native_drop = dropout_p == 0.0 or (x.is_cuda and _native.use_native(x, op="dropout") and dropout_p < 1.0)
    native_drop = native_drop and not _native.plain_fp32(x)
    fn = None
    if activation == "relu" and x.is_cuda and b is not None and native_drop:
        fn = _LinearReLU
    if activation == "gelu" and x.is_cuda and b is not None and native_drop:
        fn = _LinearGELU
    if fn is not None:
        link = arm_link(link, x)
        y = _native.apply_fn(fn, x, w, b, float(dropout_p), link)
        if link is not None and y.grad_fn is not None:
            link.first_node = weakref.ref(y.grad_fn)
        return y
    y = _lf32.linear_f32(x, w, b) if _native.plain_fp32(x) and _lf32.applies(x, w) else F.linear(x, w, b)
    y = F.gelu(y) if activation == "gelu" else F.relu(y)
    return F.dropout(y, dropout_p, True) if dropout_p > 0.0 else y


class LinearAct(torch.nn.Linear):
    """``nn.Linear`` (same parameters / keys) whose forward is ``act(x Wᵀ + b)`` via :func:`linear_act`.

    Calling it as a MODULE matters under FSDP: the unit's forward pre-hook gathers the sharded
    weight; reaching into ``.weight`` from a parent module would read a freed shard."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, activation: str = "relu", **kw):
        super().__init__(in_features, out_features, bias=bias, **kw)
        self.activation = activation

    def forward(self, x: torch.Tensor, dropout_p: float = 0.0, link=None) -> torch.Tensor:  # type: ignore[override]
        return linear_act(x, self.weight, self.bias, self.activation, dropout_p, link=link)
