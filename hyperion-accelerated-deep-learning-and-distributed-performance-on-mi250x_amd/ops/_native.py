"""Loader for the in-tree ``hyperion._C`` extension (gfx950 HIP kernels + RCCL communicator).

Policy (so GPU runs can never silently measure a PyTorch fallback):

* On a GPU box the extension MUST load: :func:`native` raises if ``_C.so`` is missing or fails
  to import (set ``HYPERION_ALLOW_TORCH_FALLBACK=1`` to opt out explicitly).
* ``HYPERION_KERNELS=torch`` forces the PyTorch reference path everywhere (A/B benchmarking).
* On CPU the kernels cannot run; ops use their PyTorch reference implementations, which are also
  the numerics oracles in ``tests/``.
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

import torch

_MOD = None
_ERR: Optional[BaseException] = None
_TRIED = False

DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _load():
    global _MOD, _ERR, _TRIED
    if _TRIED:
        return _MOD
    _TRIED = True
    try:
        _MOD = importlib.import_module("hyperion._C")
    except BaseException as e:  # noqa: BLE001 - report any load failure
        _ERR = e
        _MOD = None
    return _MOD


def backend() -> str:
    """``hyperion`` (native kernels) or ``torch`` (reference path)."""
    return os.environ.get("HYPERION_KERNELS", "hyperion").lower()


def available() -> bool:
    return _load() is not None


def native():
    """The loaded extension module; raises loudly when it should exist but does not."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "hyperion._C is not built or failed to load "
            f"({_ERR!r}); run `python -m hyperion.csrc.build` (or __graft_entry__.build())"
        )
    return m


def torch_ops() -> set:
    """Ops forced onto the PyTorch path via ``HYPERION_TORCH_OPS=bn,adam,...`` (A/B and bisection)."""
    return {o.strip() for o in os.environ.get("HYPERION_TORCH_OPS", "").split(",") if o.strip()}


def use_native(*tensors: torch.Tensor, op: Optional[str] = None) -> bool:
    """True when the native kernels should run for these tensors.

    GPU tensors + backend 'hyperion' -> native (raises if the extension is missing, unless
    HYPERION_ALLOW_TORCH_FALLBACK=1).  CPU tensors, backend 'torch', or ``op`` listed in
    ``HYPERION_TORCH_OPS`` -> reference path.
    """
    if backend() == "torch" or (op is not None and op in torch_ops()):
        return False
    if not tensors or not all(t.is_cuda for t in tensors if t is not None):
        return False
    if _load() is None:
        if os.environ.get("HYPERION_ALLOW_TORCH_FALLBACK") == "1":
            return False
        native()  # raises
    return True


_COUNTS: dict = {}


def count(op: str, n: int = 1) -> None:
    """Dispatch counter: ops record which path ran (``conv_bn_act``, ``dgrad``, ``dgrad_vendor``,
    ...), so GPU tests assert the native kernels were actually reached rather than a silent
    fallback that computes the same numbers (host-side only; one dict update per op call)."""
    _COUNTS[op] = _COUNTS.get(op, 0) + n


def counters() -> dict:
    return dict(_COUNTS)


def reset_counters() -> None:
    _COUNTS.clear()


def loaded_path() -> Optional[str]:
    m = _load()
    return getattr(m, "__file__", None) if m is not None else None
