"""LoRA linear: frozen base GEMM + low-rank update, with a regenerated dropout mask.

``y = x Wᵀ (+ b) + s · (drop(x) Aᵀ) Bᵀ``  (W frozen; A [r, in], B [out, r] trainable)

Reference: PEFT's ``lora.Linear.forward`` (dropout → ``lora_A`` → ``lora_B`` → ``* scaling`` →
add) as 4-5 separate kernels with the dropped activations stored for backward (SURVEY §2.4
"LoRA", C26).  Here one autograd function; on gfx950 (in % 64, out % 64, r % 8) every GEMM runs on
Hyperion kernels: ``t = drop(x)Aᵀ`` and the base ``x Wᵀ`` on the split-K weight-streaming kernel
with ``c·t Bᵀ`` fused into the base GEMM's reduce; in backward ``dt = c·dy B`` (split-K),
``dx = dy W + keep∘(dt A)`` (rank-r term fused into the dgrad reduce), and ``dA``/``dBᵀ`` on the
conv weight-gradient kernel at 1x1.  The math:

* forward: base GEMM (``ops.linear``: split-K weight-streaming MFMA kernel), ``t = drop(x)Aᵀ``
  ([N, r] — tiny), then ``y += c·t Bᵀ`` as a rank-r update fused into the base GEMM's reduce;
  on gfx950 drop(x) is the graph-safe counter-based kernel (``ops/dropout.py``: no stored mask,
  regenerated in backward — torch's bernoulli masks took ~4.5 ms of the Llama LoRA step);
* backward: ``dx = dy W + (c·dy B) A ∘ keep``, ``dA = (c·dy B)ᵀ drop(x)``, ``dB = c·dyᵀ t``; W
  never gets a gradient buffer.  The keep-mask is drawn in the activation dtype from the default
  device generator (one kernel; the step stays hipGraph-capturable) and ``drop(x)`` is kept for
  dA — at fine-tune shapes (hundreds of tokens) a few hundred KB per projection.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _native
from .linear import SKINNY_MAX_M, linear_dgrad, linear_fwd

def _keep_mask(x: torch.Tensor, p: float) -> torch.Tensor:
    # drawn directly in the activation dtype (one kernel; 0/1 are exact in bf16/f16) — the
    # reference path only; the native path regenerates the mask (ops/dropout.py)
    return torch.empty(x.shape, device=x.device, dtype=x.dtype).bernoulli_(1.0 - p)


def _native_ok(x2: torch.Tensor, w: torch.Tensor, a: torch.Tensor, bm: torch.Tensor) -> bool:
    """Every GEMM of the step on the gfx950 kernels: in % 64, out % 64, r % 8, same 2-byte dtype."""
    r, n_in, n_out = a.shape[0], w.shape[1], w.shape[0]
    return (x2.is_cuda and x2.dtype in (torch.bfloat16, torch.float16) and w.dtype == a.dtype == bm.dtype == x2.dtype
            and n_in % 64 == 0 and n_out % 64 == 0 and r % 8 == 0 and x2.shape[0] <= SKINNY_MAX_M
            and x2.shape[0] < (1 << 22) and w.is_contiguous() and _native.use_native(x2, op="lora"))


class _LoRAFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, a, bm, scaling, p):
        cdt = torch.get_autocast_dtype(x.device.type) if torch.is_autocast_enabled(x.device.type) else x.dtype
        xc, wc = x.to(cdt), w.to(cdt)
        ac, bc = a.to(cdt).contiguous(), bm.to(cdt).contiguous()
        x2 = xc.reshape(-1, xc.shape[-1]).contiguous()
        native = _native_ok(x2, wc, ac, bc)
        st = keep = None
        if native and p > 0:
            # graph-safe counter-based dropout: xd = x·keep/(1-p), the mask regenerated in backward
            st = _native.rng_state(x2.device)
            xd = _native.native().dropout(x2, p, st)
            c = scaling
        else:
            c = scaling / (1.0 - p) if p > 0 else scaling  # dropout's 1/(1-p) folded into the rank-r GEMM
            keep = _keep_mask(x2, p) if p > 0 else None
            xd = x2 * keep if p > 0 else x2
        if native:
            C = _native.native()
            t = C.linear_nt(xd, ac)  # [N, r]: split-K over the input features
            # base GEMM with the rank-r update fused into its split-K reduce: y = x Wᵀ + c · t Bᵀ
            y = C.linear_nt(x2, wc, U=t, V=bc, v_nr=True, beta=c)
        else:
            t = xd @ ac.t()  # [N, r]
            y = linear_fwd(x2, wc)
            y.addmm_(t, bc.t(), alpha=c)  # rank-r update in place
        if b is not None:
            y += b.to(cdt)
        ctx.save_for_backward(wc, ac, bc, t, xd, keep)
        ctx.cfg = (c, p, x.dtype, a.dtype, bm.dtype, xc.shape, native, st)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        wc, ac, bc, t, xd, keep = ctx.saved_tensors
        c, p, xdt, adt, bdt, xshape, native, st = ctx.cfg
        dy2 = dy.reshape(-1, dy.shape[-1]).to(wc.dtype).contiguous()
        dx = dA = dB = None
        M, r = t.shape
        if native:
            C = _native.native()
            dt = C.linear_nn(dy2, bc, alpha=c)  # grad of t: c · dy B  [N, r]
            if ctx.needs_input_grad[0]:
                # dx = dy W + (keep/(1-p)) ∘ (dt A): the rank-r term fused into the base dgrad's reduce,
                # the scaled mask regenerated from the forward's rng state
                mask = C.dropout(xd, p, st, mask=True) if st is not None else None
                dx = C.linear_nn(dy2, wc, U=dt, V=ac, v_nr=False, mask=mask).view(xshape).to(xdt)
            if ctx.needs_input_grad[3]:  # dA = dtᵀ drop(x): the conv weight-gradient kernel at 1x1
                dA = C.conv_wgrad(dt.view(M, r, 1, 1), xd.view(M, -1, 1, 1), 1, 1, 1, 1, 0, 0).view(r, -1).to(adt)
            if ctx.needs_input_grad[4]:  # dBᵀ = c · tᵀ dy
                dB = C.conv_wgrad(t.view(M, r, 1, 1), dy2.view(M, -1, 1, 1), 1, 1, 1, 1, 0, 0,
                                  alpha=c).view(r, -1).t().to(bdt)
            return dx, None, None, dA, dB, None, None
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
