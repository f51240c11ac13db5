"""LayerNorm / RMSNorm with an optional fused residual add (gfx950 kernels in ``layernorm.hip``).

Reference users: the two post-norm LayerNorms in every ``nn.TransformerEncoderLayer``
(SimpleTransformerLM ``distributed_utils.py:75-88``, LM-768 ``compilation_optimization.py:57-71``,
CustomTransformer ``baseline_performance.ipynb:238-249``) and HF Llama's RMSNorm (C26).

``layer_norm(x, weight, bias, eps, residual=r)`` computes ``LN(x + r)`` in one pass (post-norm:
``norm(x + dropout(sublayer(x)))``); ``return_sum=True`` also returns ``x + r`` (pre-norm residual
stream, Llama).  ``dropout_p > 0`` (training, with a residual) fuses the residual branch's dropout:
``LN(r + dropout(x))`` with the counter-based mask of ``ops.dropout`` regenerated in the kernel, and
the backward writes the dropped input's gradient ``dropout(ds)`` beside ``ds`` — the two standalone
dropout passes per norm disappear (SURVEY §2.4 LayerNorm / dropout rows).  Modules keep
``nn.LayerNorm`` state-dict keys.
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native
from . import recompute as _rc

_SUPPORTED_D = lambda d: d % 8 == 0 and d <= 4096 and ((d + 511) // 512 <= 4 or (d + 511) // 512 == 8)  # noqa: E731


def _ref(x, residual, weight, bias, eps, rms, dropout_p=0.0):
    if dropout_p > 0.0:
        x = F.dropout(x, dropout_p, True)
    s = x if residual is None else x + residual
    if rms:
        sf = s.float()
        y = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps)
        if weight is not None:
            y = y * weight.float()
        y = y.to(s.dtype)
    else:
        y = F.layer_norm(s, (s.shape[-1],), weight, bias, eps)
    return y, s


class BiasGradLink:
    """Hands a norm's branch gradient column sums to the linear layer that produced its input.

    The linear's output is the norm's ``x`` (its only consumer), so the linear's bias gradient is
    Σ_rows of the gradient the norm's backward returns for x — the LayerNorm backward kernel sums
    it while storing it (``layernorm.hip`` BSUM, combined with dγ / dβ in one launch) and parks it
    here; the linear's backward uses it when the gradient it receives IS that tensor (else it sums
    dy itself).  ``armed`` is set by the linear (it has a bias and ran the native path)."""

    __slots__ = ("armed", "db", "g", "dtype")

    def __init__(self):
        self.armed = False
        self.dtype = None  # the linear's bias dtype: the kernel writes the sums in it (no cast)
        self.db = None
        self.g = None

    def take(self, dy: torch.Tensor) -> Optional[torch.Tensor]:
        db, g = self.db, self.g
        self.db = self.g = None
        return db if (db is not None and g is dy) else None


def bias_grad_link() -> Optional[BiasGradLink]:
    return BiasGradLink() if (FUSE_BIAS_GRAD and torch.is_grad_enabled()) else None


FUSE_BIAS_GRAD = True  # A/B switch (tests)


def _will_run(ref) -> bool:
    node = ref() if ref is not None else None
    return node is not None and torch._C._will_engine_execute_node(node)


class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, rms, return_sum, dropout_p=0.0, link=None, blink=None):
        C = _native.native()
        x = x.contiguous()
        if residual is not None:
            residual = residual.contiguous().to(x.dtype)
        st = _native.rng_state(x.device) if dropout_p > 0.0 else None
        if st is not None:
            _native.count("ln_dropout")
        y, s, mean, rstd = C.ln_fwd(x, residual, weight, bias, eps, rms, dropout_p, st)
        xin = s if residual is not None else x
        ctx.rms = rms
        ctx.drop = (dropout_p, st)
        ctx.has_res = residual is not None
        ctx.link = link
        ctx.blink = blink
        ctx.save_for_backward(xin, weight, mean, rstd)
        if _rc.active():  # selective recompute: the next GEMM saves a recipe, not y
            _rc.register(y, _rc.ln_recipe(xin, weight, bias, eps, rms))
        if return_sum:
            return y, (s if residual is not None else x)
        return y

    @staticmethod
    def backward(ctx, dy, ds=None):
        xin, weight, mean, rstd = ctx.saved_tensors
        need_dw = weight is not None and ctx.needs_input_grad[2]
        need_db = ctx.needs_input_grad[3]
        p, st = ctx.drop
        blink = ctx.blink
        bsum = blink is not None and blink.armed and ctx.needs_input_grad[0]
        bdt = _native.DTYPE_CODE.get(blink.dtype, -1) if bsum else -1
        dx, dw, db, dxa, dbs = _native.native().ln_bwd(dy, xin, weight, mean, rstd, ds, need_dw, need_db, ctx.rms, p,
                                                       st, bsum, bdt)
        if bsum and dbs is not None:
            blink.db, blink.g = dbs, (dxa if p > 0.0 else dx)
        dres = dx if ctx.has_res and ctx.needs_input_grad[1] else None
        link = ctx.link
        if dres is not None and link is not None and link.armed and _will_run(link.first_node):
            # the residual input's other consumer (the block's first GEMM) adds it in its data-gradient
            # epilogue: no separate add of the two gradients of the block input
            link.dres, dres = dres, None
        return (
            dxa if p > 0.0 else dx,  # the dropped input's gradient: dropout(ds) with the forward's mask
            dres,
            dw if need_dw else None,
            db if need_db else None,
            None, None, None, None, None, None,
        )


def layer_norm(
    x: torch.Tensor,
    weight: Optional[torch.Tensor],
    bias: Optional[torch.Tensor],
    eps: float = 1e-5,
    residual: Optional[torch.Tensor] = None,
    rms: bool = False,
    return_sum: bool = False,
    dropout_p: float = 0.0,
    link=None,
    blink=None,
) -> Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
    """``LN(x + residual)`` (or RMSNorm); ``dropout_p``: ``LN(residual + dropout(x))`` — pass it only
    in training (it is applied whenever > 0)."""
    d = x.shape[-1]
    # the kernels take fp32 affine parameters or parameters in the activation dtype (a model cast
    # wholesale to bf16: FSDP mixed precision, HF-style Llama) — read as such, dγ / dβ returned in it;
    # any other mix is upcast (d elements, differentiable) rather than leave the fused path
    wdt = weight.dtype if weight is not None else (bias.dtype if bias is not None else torch.float32)
    if wdt not in (torch.float32, x.dtype) or (weight is not None and bias is not None and weight.dtype != bias.dtype):
        weight = weight.float() if weight is not None else None
        bias = bias.float() if bias is not None else None
        wdt = torch.float32
    native = (
        _native.use_native(x, op="ln")
        and x.dtype in _native.DTYPE_CODE
        and _SUPPORTED_D(d)
        and all(t is None or (t.is_contiguous() and t.data_ptr() % 16 == 0) for t in (weight, bias))
        and (residual is None or residual.shape == x.shape)
        and (dropout_p == 0.0 or (residual is not None and d <= 2048 and dropout_p < 1.0))
    )
    if native:
        if link is not None and residual is not link.src:
            link = None
        return _native.apply_fn(_LNFn, x, residual, weight, bias, eps, rms, return_sum, float(dropout_p), link, blink)
    y, s = _ref(x, residual, weight, bias, eps, rms, dropout_p)
    return (y, s) if return_sum else y


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` (same keys) with an optional fused residual input."""

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,  # type: ignore[override]
                dropout_p: float = 0.0, link=None, blink=None) -> torch.Tensor:
        """``LN(x + residual)``; ``dropout_p`` > 0: ``LN(residual + dropout(x))`` (post-norm branch)."""
        if len(self.normalized_shape) != 1:
            if dropout_p > 0.0:
                x = F.dropout(x, dropout_p, True)
            return super().forward(x if residual is None else x + residual)
        if torch.is_autocast_enabled() and x.dtype == torch.float32 and residual is not None:
            residual = residual.float()
        return layer_norm(x, self.weight, self.bias, self.eps, residual=residual, dropout_p=dropout_p, link=link,
                          blink=blink)


class RMSNorm(nn.Module):
    """RMSNorm with HF Llama's parameter name (``weight``) and fp32 statistics."""

    def __init__(self, hidden_size: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size))
        self.variance_epsilon = eps

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, return_sum: bool = False):
        return layer_norm(x, self.weight, None, self.variance_epsilon, residual=residual, rms=True,
                          return_sum=return_sum)
