"""Selective activation recompute: keep the GEMM outputs, recompute the cheap elementwise
activations in backward (reference: ``checkpoint_sequential`` /
``use_checkpoint=True`` recompute EVERY op of a block, ``memory_optimization.ipynb:194-262``).

Inside ``with selective():`` (wrapping a forward), the producers of cheap-to-rebuild activations
register a recipe for their output — LayerNorm (``LN(s)`` from the saved sum and its statistics),
the FFN's ``dropout(gelu(z))`` (from the saved pre-activation ``z`` and the dropout RNG record).
A ``saved_tensors_hooks`` pack hook then stores, for any op that saves such a tensor (or a
contiguous view of it) for backward — the next GEMM's input — the recipe instead of the tensor;
the unpack hook rebuilds it when that op's backward runs.  Nothing else changes: GEMM outputs,
attention's q/k/v/O and every tensor without a recipe are saved as usual, so the recompute is a
handful of bandwidth-bound passes per block instead of the block's whole forward.

Works under hipGraph capture (the recompute kernels are captured into the backward) and with
FSDP / DDP; recipes read only tensors the producing op saved anyway.
"""
from __future__ import annotations

import contextlib
import weakref
from typing import Callable, Dict, Optional, Tuple

import torch

_ACTIVE = 0
# storage key -> (weakref to the registered tensor, its recipe).  A freed activation's memory is
# reused by the next block's one (same key): a later register() replaces the entry, and a pack
# only takes an entry whose tensor is still alive — so the key can never name stale data.
_REG: Dict[Tuple[int, int, int, torch.dtype], Tuple["weakref.ref", "_Recipe"]] = {}
STATS = {"packed": 0, "recomputed": 0}


def active() -> bool:
    # (no grad-mode check: autograd Functions run their forward under no_grad; selective() is only
    # entered when the forward records a graph)
    return _ACTIVE > 0


def _key(t: torch.Tensor):
    return (t.untyped_storage().data_ptr(), t.storage_offset(), t.numel(), t.dtype)


def register(t: torch.Tensor, fn: Callable[[], torch.Tensor]) -> None:
    """``fn()`` rebuilds ``t`` (same values up to rounding, same dtype and numel) in backward."""
    if active() and t.is_contiguous():
        _REG[_key(t)] = (weakref.ref(t), _Recipe(fn, t.shape))


class _Recipe:
    __slots__ = ("fn", "shape", "out")

    def __init__(self, fn, shape):
        self.fn, self.shape, self.out = fn, shape, None

    def get(self, shape) -> torch.Tensor:
        if self.out is None:
            STATS["recomputed"] += 1
            self.out = self.fn()
        return self.out.view(shape)


def _pack(t: torch.Tensor):
    if not t.is_contiguous():
        return t
    e = _REG.get(_key(t))
    if e is None or e[0]() is None:  # no recipe, or its tensor died (storage may be reused)
        return t
    STATS["packed"] += 1
    return (e[1], t.shape)  # every save of one live tensor shares its recipe (rebuilt once)


def _unpack(p):
    if isinstance(p, tuple) and len(p) == 2 and isinstance(p[0], _Recipe):
        return p[0].get(p[1])
    return p


@contextlib.contextmanager
def selective(enabled: bool = True):
    """Forward region whose registered activations are rebuilt in backward instead of saved."""
    global _ACTIVE
    if not (enabled and torch.is_grad_enabled()):
        yield
        return
    _ACTIVE += 1
    try:
        with torch.autograd.graph.saved_tensors_hooks(_pack, _unpack):
            yield
    finally:
        _ACTIVE -= 1
        if _ACTIVE == 0:
            _REG.clear()


def ln_recipe(xin: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor], eps: float,
              rms: bool) -> Callable[[], torch.Tensor]:
    def fn():
        from . import _native

        y, _s, _m, _r = _native.native().ln_fwd(xin, None, weight, bias, eps, rms, 0.0, None)
        return y

    return fn
