"""Fused linear + softmax cross-entropy (the LM head and its loss as one op).

Reference: ``logits = fc(x)`` then ``nn.CrossEntropyLoss(ignore_index=pad)`` over V = 50257 in
every LM trainer (``02_development/distributed_utils.py:161,175-177``, ``core_framework.ipynb:
243-262``, ``mixed_precision.ipynb:121-145``) — the logits GEMM dominates LM compute (≈105 GFLOP
forward at 4064 tokens) and PyTorch materialises fp32 log-softmax and its gradient.

Hyperion computes the loss AND all three gradients inside the forward.  Two schedules (gfx950,
bf16/f16):

**Materialised** (default while the [N, V] logits take at most HYPERION_CE_MATERIALIZE_MB,
8 GiB — GPT-2 b16: 206 MB, LM-256 b32: 408 MB of a 288 GB device): the logits GEMM writes bf16
logits once (hipBLASLt, rows padded to a multiple of 8 classes so every row is 16-byte aligned);
ce_fwd_bwd (cross_entropy.hip, the register-resident variant: one read + one write per
logit) adds the bias, takes the loss and overwrites the logits with dz in place; then
dX = dz W on the tiled MFMA kernel with split-K (ops.gemm.mm_nn on the 64-aligned class
range, the odd tail as a rank-17 update), dW = dzᵀ X on hipBLASLt and db as column sums.
Three GEMMs instead of four (no logits recompute): 0.66 vs 1.30 ms for GPT-2-small b16 and
0.68 vs 1.48 ms for LM-256 b32 (scripts/ce_bench.py, profiles/r04/ce_bench_lm_head.json).

**No-logits** (above that budget; never stores the [N, V] logits, E % 64 == 0):

1. ``linear_ce_lse`` — the logits GEMM on the MFMA implicit-GEMM kernel with a log-sum-exp
   epilogue (``conv_igemm.hip`` EPI 1): every 128 x 64 tile reduces its accumulators to per-row
   (max, Σexp) partials and captures the target logit; a one-wave-per-row combine
   (``cross_entropy.hip``) gives lse and the per-row losses.  No logits tensor exists;
2. per vocabulary chunk (``chunk`` classes, default 8192): ``linear_ce_grad`` recomputes the
   chunk's logits on the same kernel and its epilogue writes dz = (exp(z − lse) − onehot) /
   n_valid straight from the accumulators (EPI 2); then ``dx += dz W_c`` and ``dW_c = dzᵀ x``
   (vendor GEMMs) and ``db_c = Σ dz`` (column sums).  Peak extra memory is one [N, chunk] dz
   block instead of the [N, V] logits (LM-256: 65 MB instead of 408 MB).

Backward then only scales the saved gradients by the incoming scalar.  ``n_valid`` (non-ignored
tokens) stays on the device, so the op has no host sync and is hipGraph-capturable.  Elsewhere
(CPU, fp32) the reference path materializes ``z`` (in row chunks above ``max_logits_bytes``) and
runs ``ce_fwd_bwd`` / the PyTorch oracle on it.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import _native

import os

DEFAULT_MAX_LOGITS_BYTES = 4 << 30
# The fused path's dz block is at most CE_BLOCK_BYTES: the vocabulary is cut into the fewest equal
# 64-class-aligned chunks that fit (LM-256, 4064 x 50257 bf16 = 408 MB of logits: 2 chunks; fewer,
# larger chunks keep the dX / dW GEMMs efficient).  HYPERION_CE_CHUNK forces a class count.
CE_BLOCK_BYTES = int(os.environ.get("HYPERION_CE_BLOCK_MB", "256")) << 20
CE_CHUNK = int(os.environ.get("HYPERION_CE_CHUNK", "0"))
# logits budget of the materialised schedule (module docstring); 0 forces the no-logits schedule.
# Default: 1/32 of the device's HBM (9 GiB on a 288 GB MI355X, 2 GiB on a 64 GB MI250X GCD), and
# never more than half of what is free at the call
_CE_MAT_ENV = os.environ.get("HYPERION_CE_MATERIALIZE_MB")
CE_MATERIALIZE_BYTES = int(_CE_MAT_ENV) << 20 if _CE_MAT_ENV is not None else None
_HBM_BUDGET = {}


_SCHEDULE = {}  # (device, N, V-padded, element size) -> materialise the logits?


def _materialize_budget(dev: torch.device) -> int:
    if CE_MATERIALIZE_BYTES is not None:
        return CE_MATERIALIZE_BYTES
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _HBM_BUDGET:
        _HBM_BUDGET[idx] = torch.cuda.get_device_properties(idx).total_memory // 32
    budget = _HBM_BUDGET[idx]
    if torch.cuda.is_current_stream_capturing():
        return budget  # no free-memory query inside a capture; the graph pool was sized eagerly
    free, _ = torch.cuda.mem_get_info(idx)
    # blocks the caching allocator holds but does not use are free for this op too
    free += torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
    return min(budget, free // 2)


def _materialize(dev: torch.device, N: int, V: int, elt: int) -> bool:
    """The schedule (materialised logits or not) is decided ONCE per (device, shape, dtype) on the
    first call and reused: a per-call free-memory check could flip it between steps (different
    numerics and memory) or pick, under hipGraph capture, a logits buffer that eager warm-up
    never sized."""
    vp = -(-V // 8) * 8
    if CE_MATERIALIZE_BYTES is not None:  # an explicit budget: a fixed rule, nothing to cache
        return N * vp * elt <= CE_MATERIALIZE_BYTES
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, N, vp, elt)
    if key not in _SCHEDULE:
        _SCHEDULE[key] = N * key[2] * elt <= _materialize_budget(dev)
    return _SCHEDULE[key]


def _ce_chunk(N: int, V: int, elt: int) -> int:
    if CE_CHUNK > 0:
        return CE_CHUNK
    n = max(1, -(-N * V * elt // CE_BLOCK_BYTES))
    return -(-(-(-V // n)) // 64) * 64


def _compute_dtype(x: torch.Tensor, w: torch.Tensor) -> torch.dtype:
    if torch.is_autocast_enabled(x.device.type):
        return torch.get_autocast_dtype(x.device.type)
    return x.dtype if x.dtype == w.dtype else torch.promote_types(x.dtype, w.dtype)


def _ce_chunk_reference(z: torch.Tensor, t: torch.Tensor, scale: torch.Tensor, ignore_index: int):
    """PyTorch oracle of the in-place kernel: returns (loss_rows, dz)."""
    zf = z.float()
    lse = torch.logsumexp(zf, dim=-1)
    valid = t != ignore_index
    tc = torch.where(valid, t, torch.zeros_like(t))
    zt = zf.gather(1, tc[:, None]).squeeze(1)
    loss = torch.where(valid, lse - zt, torch.zeros_like(lse))
    p = torch.exp(zf - lse[:, None])
    p.scatter_add_(1, tc[:, None], -torch.ones_like(zt)[:, None])
    dz = p * (scale * valid.float())[:, None]
    return loss, dz.to(z.dtype)


class _FusedLinearCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, target, ignore_index, max_bytes):
        cdt = _compute_dtype(x, weight)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).to(cdt)
        t = target.reshape(-1)
        N, V = x2.shape[0], weight.shape[0]
        w = weight.to(cdt)
        b = bias.to(cdt) if bias is not None else None
        n_valid = (t != ignore_index).sum().to(torch.float32).clamp_min(1.0)
        scale = (1.0 / n_valid).reshape(1)
        native = _native.use_native(x2, op="ce") and cdt in _native.DTYPE_CODE
        if native and cdt in (torch.bfloat16, torch.float16) and x2.is_cuda:
            if _materialize(x2.device, N, V, x2.element_size()):
                return _FusedLinearCE._materialized(ctx, x, x2, w, bias, t, ignore_index, scale, shape)
            if x2.shape[1] % 64 == 0:
                return _FusedLinearCE._fused(ctx, x, x2, w, bias, t, ignore_index, scale, n_valid, shape)
        rows = max(1, min(N, max_bytes // max(1, V * x2.element_size())))
        dx = torch.empty_like(x2)
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        dw = None
        db = None
        loss_sum = torch.zeros((), dtype=torch.float32, device=x.device)
        chunked = rows < N
        for r0 in range(0, N, rows):
            xc, tc = x2[r0 : r0 + rows], t[r0 : r0 + rows].contiguous()
            z = F.linear(xc, w, b)
            if native:
                loss_rows, _ = _native.native().ce_fwd_bwd(z, tc, scale, 1.0, int(ignore_index), True)
                dz = z
            else:
                loss_rows, dz = _ce_chunk_reference(z, tc, scale, ignore_index)
            loss_sum = loss_sum + loss_rows.sum()
            torch.mm(dz, w, out=dx[r0 : r0 + rows])
            if need_w:
                g = dz.t().mm(xc)
                if not chunked:
                    dw = g
                else:
                    dw = g.float() if dw is None else dw.add_(g.float())
            if need_b:
                s = dz.sum(0, dtype=torch.float32)
                db = s if db is None else db.add_(s)
        loss = loss_sum * scale.reshape(())
        ctx.save_for_backward(dx.view(shape), dw if dw is not None else torch.empty(0),
                              db if db is not None else torch.empty(0))
        ctx.meta = (x.dtype, weight.dtype, None if bias is None else bias.dtype, need_w, need_b)
        return loss

    @staticmethod
    def _materialized(ctx, x, x2, w, bias, t, ignore_index, scale, shape):
        """bf16 logits once, CE in place, then the two backward GEMMs on dz (module docstring)."""
        from .gemm import lm_head_dx, lm_head_logits, mm_nn, mm_tn

        C = _native.native()
        _native.count("linear_ce_materialized")
        x2 = x2.contiguous()
        w = w.contiguous()
        t = t.contiguous()
        N, V = x2.shape[0], w.shape[0]
        Vp = -(-V // 8) * 8
        zb = torch.empty(N, Vp, dtype=x2.dtype, device=x2.device)
        z = zb[:, :V]  # 16-byte aligned rows
        if not lm_head_logits(x2, w, zb):
            torch.mm(x2, w.t(), out=z)
            if Vp > V:
                zb[:, V:].zero_()  # the class-reducing dX GEMM reads the row padding
        b32 = None
        if bias is not None:
            b32 = bias.detach().float().contiguous()
            if b32.data_ptr() % 16:
                b32 = b32.clone()
        loss_rows, _ = C.ce_fwd_bwd(z, t, scale, 1.0, int(ignore_index), True, b32)  # z <- dz
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        dx = None
        if ctx.needs_input_grad[0]:
            dx = lm_head_dx(zb, w)
            if dx is None:
                Vm = V // 64 * 64
                dx = mm_nn(zb[:, :Vm], w[:Vm]) if Vm > 0 else None
                if dx is None:
                    dx = torch.mm(z, w)
                elif Vm < V:
                    dx.addmm_(z[:, Vm:], w[Vm:])  # the odd class tail (rank V - Vm)
        dw = None
        if need_w:
            dwp = mm_tn(zb, x2)  # [Vp, E]: the padding classes' rows are dropped
            dw = dwp[:V] if dwp is not None else torch.mm(z.t(), x2)
        db = C.column_sum(zb, torch.float32)[:V] if need_b else None
        loss = loss_rows.sum() * scale.reshape(())
        ctx.save_for_backward(dx.view(shape) if dx is not None else torch.empty(0),
                              dw if dw is not None else torch.empty(0), db if db is not None else torch.empty(0))
        ctx.meta = (x.dtype, w.dtype, None if bias is None else bias.dtype, need_w, need_b)
        return loss

    @staticmethod
    def _fused(ctx, x, x2, w, bias, t, ignore_index, scale, n_valid, shape):
        """The no-logits path (module docstring): LSE pass, then per-chunk gradient passes."""
        C = _native.native()
        _native.count("linear_ce_fused")
        x2 = x2.contiguous()
        w = w.contiguous()
        b32 = bias.float().contiguous() if bias is not None else None
        t = t.contiguous()
        N, V = x2.shape[0], w.shape[0]
        lse, loss_rows = C.linear_ce_lse(x2, w, b32, t, int(ignore_index))
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        dx32 = None
        dw = torch.empty_like(w) if need_w else None
        db = torch.empty(V, dtype=torch.float32, device=x2.device) if need_b else None
        chunk = _ce_chunk(N, V, x2.element_size())
        for c0 in range(0, V, chunk):
            n = min(chunk, V - c0)
            dz = C.linear_ce_grad(x2, w, b32, t, int(ignore_index), lse, scale, c0, n)  # [N, ceil8(n)]
            dzv = dz[:, :n]
            wc = w[c0:c0 + n]
            # dX accumulates over the chunks in fp32 inside the GEMM (bf16 inputs, fp32 output)
            dx32 = (torch.mm(dzv, wc, out_dtype=torch.float32) if dx32 is None
                    else torch.addmm(dx32, dzv, wc, out_dtype=torch.float32))
            if need_w:
                torch.mm(dzv.t(), x2, out=dw[c0:c0 + n])
            if need_b:
                db[c0:c0 + n] = C.column_sum(dz, torch.float32)[:n]
        loss = loss_rows.sum() * scale.reshape(())
        ctx.save_for_backward(dx32.to(x2.dtype).view(shape), dw if dw is not None else torch.empty(0),
                              db if db is not None else torch.empty(0))
        ctx.meta = (x.dtype, w.dtype, None if bias is None else bias.dtype, need_w, need_b)
        return loss

    @staticmethod
    def backward(ctx, g):
        dx, dw, db = ctx.saved_tensors
        xdt, wdt, bdt, need_w, need_b = ctx.meta
        gx = (dx * g.to(dx.dtype)).to(xdt) if ctx.needs_input_grad[0] else None
        gw = (dw * g.to(dw.dtype)).to(wdt) if need_w else None
        gb = (db * g.to(db.dtype)).to(bdt) if need_b else None
        return gx, gw, gb, None, None, None


def fused_linear_cross_entropy(
    x: torch.Tensor,
    weight: torch.Tensor,
    bias: Optional[torch.Tensor],
    target: torch.Tensor,
    ignore_index: int = -100,
    max_logits_bytes: int = DEFAULT_MAX_LOGITS_BYTES,
) -> torch.Tensor:
    """Mean cross-entropy of ``x @ weight.T + bias`` against ``target`` over non-ignored rows.

    Equivalent to ``F.cross_entropy(F.linear(x, weight, bias).view(-1, V), target.view(-1),
    ignore_index=ignore_index)`` without materialising fp32 log-probabilities.
    """
    if not torch.is_grad_enabled() or not (x.requires_grad or weight.requires_grad):
        z = F.linear(x, weight, bias)
        return F.cross_entropy(z.reshape(-1, z.shape[-1]).float(), target.reshape(-1), ignore_index=ignore_index)
    return _FusedLinearCE.apply(x, weight, bias, target, int(ignore_index), int(max_logits_bytes))


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Plain CE on materialised logits (small class counts, e.g. CIFAR's 10)."""
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), target.reshape(-1), ignore_index=ignore_index)


class LinearCrossEntropy(torch.nn.Linear):
    """``nn.Linear`` (same keys) whose call with ``target=`` returns the fused mean CE loss.

    Running the head through ``__call__`` (instead of reading ``.weight`` from outside) keeps
    module hooks — FSDP's parameter gather, activation checkpointing — working on the LM head.
    """

    def forward(self, x: torch.Tensor, target: Optional[torch.Tensor] = None,  # type: ignore[override]
                ignore_index: int = -100) -> torch.Tensor:
        if target is None:
            return F.linear(x, self.weight, self.bias)
        return fused_linear_cross_entropy(x, self.weight, self.bias, target, ignore_index=ignore_index)
