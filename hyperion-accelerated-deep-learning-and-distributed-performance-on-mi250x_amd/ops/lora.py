"""LoRA linear: frozen base GEMM + low-rank update, with a regenerated dropout mask.

``y = x Wᵀ (+ b) + s · (drop(x) Aᵀ) Bᵀ``  (W frozen; A [r, in], B [out, r] trainable)

Reference: PEFT's ``lora.Linear.forward`` (dropout → ``lora_A`` → ``lora_B`` → ``* scaling`` →
add) as 4-5 separate kernels with the dropped activations stored for backward (SURVEY §2.4
"LoRA", C26).  Here one autograd function:

* forward: base GEMM (hipBLASLt), ``t = s·drop(x)Aᵀ`` ([N, r] — tiny), then ``y += t Bᵀ`` as an
  in-place rank-r update (``addmm_`` with beta=1: no second [N, out] tensor);
* backward: ``dx = dy W + (dy B · s) A∘mask``, ``dA = (s·dy B)ᵀ drop(x)``, ``dB = dyᵀ t``; W never
  gets a gradient buffer.  The dropout keep-mask is drawn from the default device generator (so the
  whole step stays hipGraph-capturable) and kept as uint8 for backward — at fine-tune shapes
  (hundreds of tokens) that is a few hundred KB per projection.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

def _keep_mask(x: torch.Tensor, p: float) -> torch.Tensor:
    return torch.empty(x.shape, device=x.device, dtype=torch.float32).bernoulli_(1.0 - p).to(torch.uint8)


def _apply(x: torch.Tensor, keep: torch.Tensor, p: float) -> torch.Tensor:
    return x * keep.to(x.dtype) * (1.0 / (1.0 - p))


class _LoRAFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, a, bm, scaling, p):
        cdt = torch.get_autocast_dtype(x.device.type) if torch.is_autocast_enabled(x.device.type) else x.dtype
        xc, wc = x.to(cdt), w.to(cdt)
        ac, bc = a.to(cdt), bm.to(cdt)
        keep = _keep_mask(xc, p) if p > 0 else None
        xd = _apply(xc, keep, p) if p > 0 else xc
        x2 = xc.reshape(-1, xc.shape[-1])
        t = (xd.reshape(-1, xd.shape[-1]) @ ac.t()) * scaling  # [N, r]
        y = F.linear(x2, wc, b.to(cdt) if b is not None else None)
        y.addmm_(t, bc.t())  # rank-r update in place
        ctx.save_for_backward(xc, wc, ac, bc, t, keep)
        ctx.cfg = (scaling, p, x.dtype, a.dtype, bm.dtype)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        xc, wc, ac, bc, t, keep = ctx.saved_tensors
        scaling, p, xdt, adt, bdt = ctx.cfg
        dy2 = dy.reshape(-1, dy.shape[-1]).to(wc.dtype)
        dx = dA = dB = None
        dt = (dy2 @ bc) * scaling  # [N, r]
        if ctx.needs_input_grad[0]:
            dxd = dt @ ac  # grad wrt drop(x)
            if p > 0:
                dxd = _apply(dxd, keep.reshape(dxd.shape), p)
            dx = torch.addmm(dxd, dy2, wc).view(xc.shape).to(xdt)
        if ctx.needs_input_grad[3]:
            xd = _apply(xc, keep, p) if p > 0 else xc
            dA = (dt.t() @ xd.reshape(-1, xd.shape[-1])).to(adt)
        if ctx.needs_input_grad[4]:
            dB = (dy2.t() @ t).to(bdt)
        return dx, None, None, dA, dB, None, None


def lora_linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], a: torch.Tensor, bm: torch.Tensor,
                scaling: float, p: float = 0.0) -> torch.Tensor:
    return _LoRAFn.apply(x, w, b, a, bm, float(scaling), float(p))


def lora_linear_reference(x, w, b, a, bm, scaling, mask=None):
    xd = x if mask is None else x * mask
    return F.linear(x, w, b) + F.linear(F.linear(xd, a), bm) * scaling
