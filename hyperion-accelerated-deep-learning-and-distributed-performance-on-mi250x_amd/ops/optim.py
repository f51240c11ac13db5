"""Fused multi-tensor Adam / AdamW on gfx950 (one launch for every parameter).

Reference optimizers: ``optim.Adam(lr=1e-3)`` in the baseline step benchmark
(``baseline_performance.ipynb:282``) and ``AdamW`` in every trainer (``distributed_utils.py:161,
232,334,503``).  torch's implementation launches a chain of ``_foreach_*`` kernels per parameter
group chunk; ``FusedAdam`` runs ``adam_mt_k`` once, reading step / loss-scale / found-inf from
device memory so the step can be captured in a hipGraph and skipped on overflow without a host
sync (GradScaler semantics).

Low-precision parameters (bf16/fp16 — "compute copies") get an fp32 master copy in the optimizer
state; the kernel updates the master and rewrites the compute copy in the same pass.  This lets a
model run its convolutions/GEMMs on bf16 weights directly (no per-forward autocast weight casts,
no bf16→fp32 grad casts in backward) while the optimizer math stays in fp32.

Also provides multi-tensor global-norm clipping that takes the norm over *all* gradient shards
(all-reduced when a process group is given) — the reference clipped only the local FSDP shard
(``distributed_utils.py:351,522``).
"""
from __future__ import annotations

import math
import weakref
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

from . import _native
from .multi_tensor import TableCache


def grad_of(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The gradient the optimizer should consume: ``p.main_grad`` (an fp32 reduced-gradient view
    that data-parallel wrappers attach to low-precision parameters, ``parallel/ddp.py``) when set,
    else ``p.grad``."""
    g = getattr(p, "main_grad", None)
    return g if g is not None else p.grad


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same element order in memory (strides of size-1 dims are irrelevant: a [K, C, 1, 1] weight is
    'contiguous' and 'channels-last' at once, and autograd may hand back either stride set)."""
    return a.shape == b.shape and all(sa == sb for sa, sb, n in zip(a.stride(), b.stride(), a.shape) if n > 1)


class FusedAdam(torch.optim.Optimizer):
    def __init__(
        self,
        params: Iterable,
        lr: float = 1e-3,
        betas=(0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.0,
        adamw: bool = False,
        zero_grad_in_step: bool = False,
    ):
        """``zero_grad_in_step``: the kernel writes zeros over each gradient as it consumes it, so
        ``zero_grad(set_to_none=False)`` before the next backward is free (one fill kernel per
        parameter saved — 256 launches per step for Llama LoRA under hipGraph capture)."""
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=adamw)
        super().__init__(params, defaults)
        self.zero_grad_in_step = zero_grad_in_step
        self._tables = TableCache()
        self._step_t: Optional[torch.Tensor] = None
        self._host_step = 0
        # optional device scalars set by the AMP scaler
        self.inv_scale: Optional[torch.Tensor] = None
        self.found_inf: Optional[torch.Tensor] = None
        # a global-norm clip coefficient left for this step by clip_grad_norm_(defer_to=self): the
        # kernel applies it while it reads the gradients (no separate scaling pass); consumed by step()
        self.clip_coef: Optional[torch.Tensor] = None

    def _state(self, p: torch.Tensor):
        st = self.state[p]
        if not st:
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.preserve_format)
            if p.dtype != torch.float32:
                st["master"] = p.detach().to(torch.float32, memory_format=torch.preserve_format).clone()
        return st

    def zero_grad(self, set_to_none: bool = True) -> None:
        if self.zero_grad_in_step and not set_to_none:
            return  # the last step already zeroed every gradient it consumed
        super().zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._host_step += 1
        first = next((p for g in self.param_groups for p in g["params"] if grad_of(p) is not None), None)
        if first is None:
            return loss
        native = _native.use_native(first, op="adam")
        inv_scale = self.inv_scale
        if self.clip_coef is not None:
            inv_scale = self.clip_coef if inv_scale is None else self.clip_coef * inv_scale
            self.clip_coef = None
        if native:
            if self._step_t is None or self._step_t.device != first.device:
                self._step_t = torch.full((), float(self._host_step - 1), dtype=torch.float32, device=first.device)
            self._step_t.add_(1.0)
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if grad_of(p) is not None]
            # partition by (param dtype, grad dtype): one launch per partition (an fp32 main_grad
            # of a bf16 parameter is its own partition: fp32 grads, bf16 params + fp32 masters)
            parts = {}
            for p in params:
                parts.setdefault((p.dtype, grad_of(p).dtype), []).append(p)
            for (pdt, gdt), ps in parts.items():
                sts = [self._state(p) for p in ps]
                gs = [grad_of(p) for p in ps]
                ms = [s["exp_avg"] for s in sts]
                vs = [s["exp_avg_sq"] for s in sts]
                masters = [s["master"] for s in sts] if pdt != torch.float32 else None
                ok = native and pdt in _native.DTYPE_CODE and gdt in _native.DTYPE_CODE and all(
                    (g.stride() == p.stride() and m.stride() == p.stride() and p.is_contiguous())  # fast path
                    or (_dense(p) and _dense(g) and _same_layout(p, g) and _same_layout(p, m))
                    for p, g, m in zip(ps, gs, ms)
                )
                if ok:
                    groups = [ps, gs, ms, vs] + ([masters] if masters is not None else [])
                    try:
                        tab = self._tables.get(f"adam{gi}_{pdt}_{gdt}", groups)
                    except ValueError:  # misaligned tensor -> reference path
                        ok = False
                if ok:
                    lr = group["lr"]
                    lr_t = lr if isinstance(lr, torch.Tensor) else None
                    b1, b2 = group["betas"]
                    _native.native().adam_mt(
                        tab.ptrs, tab.sizes, tab.blocks, tab.T, tab.chunk,
                        float(lr) if lr_t is None else 0.0, b1, b2, group["eps"], group["weight_decay"],
                        bool(group["adamw"]), lr_t, self._step_t, inv_scale, self.found_inf,
                        _native.DTYPE_CODE[gdt], _native.DTYPE_CODE[pdt], bool(self.zero_grad_in_step),
                    )
                else:
                    self._reference_step(group, ps, gs, ms, vs, masters, inv_scale)
                    if self.zero_grad_in_step:
                        for g in gs:
                            g.zero_()
        return loss

    def _reference_step(self, group, ps, gs, ms, vs, masters=None, inv_scale=None):
        """PyTorch reference (CPU / fallback); identical math to the kernel."""
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # the host-side step count would be baked into the graph (frozen bias correction)
            raise RuntimeError("FusedAdam: reference path reached during hipGraph capture (grad/param layouts "
                               "or dtypes outside the fused kernel's envelope)")
        if self.found_inf is not None and float(self.found_inf) != 0.0:
            return
        b1, b2 = group["betas"]
        lr = float(group["lr"])
        wd = group["weight_decay"]
        step = self._host_step
        bc1 = 1 - b1**step
        bc2_sqrt = math.sqrt(1 - b2**step)
        inv = float(inv_scale) if inv_scale is not None else 1.0
        for i, (p, g, m, v) in enumerate(zip(ps, gs, ms, vs)):
            w = masters[i] if masters is not None else p
            g = g.float() * inv
            if group["adamw"]:
                w.mul_(1 - lr * wd)
            elif wd != 0:
                g = g.add(w, alpha=wd)
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / bc2_sqrt).add_(group["eps"])
            w.addcdiv_(m, denom, value=-lr / bc1)
            if masters is not None:
                p.copy_(w)

    def state_dict(self):
        sd = super().state_dict()
        sd["hyperion_step"] = self._host_step
        return sd

    def load_state_dict(self, state_dict):
        state_dict = dict(state_dict)
        self._host_step = int(state_dict.pop("hyperion_step", 0))
        super().load_state_dict(state_dict)
        self._step_t = None
        # the table cache is kept: tables a captured graph uses stay pinned; new state tensors
        # simply key new tables


def FusedAdamW(params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
    return FusedAdam(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=True)


# clip tables per model: keyed (weakly) by the first parameter, so two same-shaped models never
# share -- and, once captured, never re-point -- each other's pointer table
# (a WeakKeyDictionary cannot hold tensors: its weakref keys compare their referents with the
# elementwise Tensor.__eq__ on a hash-bucket collision)
_clip_tables: "dict[int, tuple]" = {}


def _clip_cache(p0: torch.Tensor) -> TableCache:
    ent = _clip_tables.get(id(p0))
    if ent is None or ent[0]() is not p0:
        key = id(p0)
        ref = weakref.ref(p0, lambda _r, k=key: _clip_tables.pop(k, None))
        ent = (ref, TableCache())
        _clip_tables[key] = ent
    return ent[1]


@torch.no_grad()
def clip_grad_norm_(
    parameters: Iterable[torch.Tensor],
    max_norm: float,
    group: Optional["dist.ProcessGroup"] = None,
    sharded: bool = False,
    defer_to: Optional[FusedAdam] = None,
) -> torch.Tensor:
    """Clip by the global L2 norm.

    ``sharded=True``: each rank holds a disjoint shard of the gradients (FSDP); the squared norm
    is all-reduced over ``group`` before clipping — the reference's ``clip_grad_norm_`` on FSDP
    modules skipped this and clipped by the local shard norm.
    ``defer_to``: a FusedAdam whose next ``step()`` applies the clip coefficient as it reads the
    gradients (one pass over them fewer); the ``.grad`` tensors themselves are left unclipped.
    """
    params = [p for p in parameters if grad_of(p) is not None]
    grads: List[torch.Tensor] = [grad_of(p) for p in params]
    if not grads:
        return torch.zeros(())
    dev = grads[0].device
    native = _native.use_native(grads[0], op="clip") and all(_dense(g) and g.dtype == grads[0].dtype for g in grads)
    if native:
        try:
            tab = _clip_cache(params[0]).get("clip", [grads])
        except ValueError:
            native = False
    if native:
        code = _native.DTYPE_CODE[grads[0].dtype]
        total_sq = _native.native().sumsq_mt(tab.ptrs, tab.sizes, tab.blocks, tab.chunk, code)
    else:
        total_sq = torch.zeros(1, device=dev, dtype=torch.float32)
        for g in grads:
            total_sq += g.float().pow(2).sum()
    if sharded and dist.is_available() and dist.is_initialized():
        from ..train import segments as _seg

        _seg.eager(lambda: dist.all_reduce(total_sq, group=group))  # a hole of a segmented capture
    if defer_to is not None:
        defer_to.clip_coef = (max_norm / (total_sq.reshape(1).sqrt() + 1e-6)).clamp(max=1.0)
    elif native:
        _native.native().clip_mt(tab.ptrs, tab.sizes, tab.blocks, tab.chunk, total_sq, float(max_norm), code)
    else:
        coef = (max_norm / (total_sq.sqrt() + 1e-6)).clamp(max=1.0)
        for g in grads:
            g.mul_(coef.to(g.dtype))
    return total_sq.sqrt().reshape(())
