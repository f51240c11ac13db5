"""LoRA linear: frozen base GEMM + low-rank update, with a regenerated dropout mask.

``y = x Wᵀ (+ b) + s · (drop(x) Aᵀ) Bᵀ``  (W frozen; A [r, in], B [out, r] trainable)

Reference: PEFT's ``lora.Linear.forward`` (dropout → ``lora_A`` → ``lora_B`` → ``* scaling`` →
add) as 4-5 separate kernels with the dropped activations stored for backward (SURVEY §2.4
"LoRA", C26).  Here one autograd function:

* forward: base GEMM (``ops.linear``: split-K weight-streaming MFMA kernel), ``t = drop(x)Aᵀ``
  ([N, r] — tiny), then ``y += c·t Bᵀ`` with c = s/(1-p) (the dropout rescale folded into the
  GEMM's alpha) as an in-place rank-r update (``addmm_``: no second [N, out] tensor);
* backward: ``dx = dy W + (c·dy B) A ∘ keep``, ``dA = (c·dy B)ᵀ drop(x)``, ``dB = c·dyᵀ t``; W
  never gets a gradient buffer.  The keep-mask is drawn in the activation dtype from the default
  device generator (one kernel; the step stays hipGraph-capturable) and ``drop(x)`` is kept for
  dA — at fine-tune shapes (hundreds of tokens) a few hundred KB per projection.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .linear import linear_dgrad, linear_fwd

def _keep_mask(x: torch.Tensor, p: float) -> torch.Tensor:
    # drawn directly in the activation dtype (one kernel; 0/1 are exact in bf16/f16)
    return torch.empty(x.shape, device=x.device, dtype=x.dtype).bernoulli_(1.0 - p)


class _LoRAFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, a, bm, scaling, p):
        cdt = torch.get_autocast_dtype(x.device.type) if torch.is_autocast_enabled(x.device.type) else x.dtype
        xc, wc = x.to(cdt), w.to(cdt)
        ac, bc = a.to(cdt), bm.to(cdt)
        c = scaling / (1.0 - p) if p > 0 else scaling  # dropout's 1/(1-p) folded into the rank-r GEMM
        x2 = xc.reshape(-1, xc.shape[-1])
        keep = _keep_mask(x2, p) if p > 0 else None
        xd = x2 * keep if p > 0 else x2
        t = xd @ ac.t()  # [N, r]
        y = linear_fwd(x2, wc)  # weight-streaming split-K kernel at fine-tune token counts
        if b is not None:
            y += b.to(cdt)
        y.addmm_(t, bc.t(), alpha=c)  # rank-r update in place
        ctx.save_for_backward(wc, ac, bc, t, xd, keep)
        ctx.cfg = (c, p, x.dtype, a.dtype, bm.dtype, xc.shape)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        wc, ac, bc, t, xd, keep = ctx.saved_tensors
        c, p, xdt, adt, bdt, xshape = ctx.cfg
        dy2 = dy.reshape(-1, dy.shape[-1]).to(wc.dtype)
        dx = dA = dB = None
        dt = torch.mm(dy2, bc).mul_(c)  # grad of t: [N, r]
        if ctx.needs_input_grad[0]:
            dx = linear_dgrad(dy2, wc)
            dxd = dt @ ac  # grad wrt drop(x)
            if p > 0:
                dx.addcmul_(dxd, keep)
            else:
                dx += dxd
            dx = dx.view(xshape).to(xdt)
        if ctx.needs_input_grad[3]:
            dA = (dt.t() @ xd).to(adt)
        if ctx.needs_input_grad[4]:
            dB = torch.mm(dy2.t(), t).mul_(c).to(bdt)
        return dx, None, None, dA, dB, None, None


def lora_linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], a: torch.Tensor, bm: torch.Tensor,
                scaling: float, p: float = 0.0) -> torch.Tensor:
    return _LoRAFn.apply(x, w, b, a, bm, float(scaling), float(p))


def lora_linear_reference(x, w, b, a, bm, scaling, mask=None):
    xd = x if mask is None else x * mask
    return F.linear(x, w, b) + F.linear(F.linear(xd, a), bm) * scaling
