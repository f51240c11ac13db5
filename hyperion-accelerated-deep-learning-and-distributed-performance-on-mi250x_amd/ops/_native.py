"""Loader for the in-tree ``hyperion._C`` extension (gfx950 HIP kernels + RCCL communicator).

Policy (so GPU runs can never silently measure a PyTorch fallback):

* On a GPU box the extension MUST load: :func:`native` raises if ``_C.so`` is missing or fails
  to import (set ``HYPERION_ALLOW_TORCH_FALLBACK=1`` to opt out explicitly).
* ``HYPERION_KERNELS=torch`` forces the PyTorch reference path everywhere (A/B benchmarking).
* On CPU the kernels cannot run; ops use their PyTorch reference implementations, which are also
  the numerics oracles in ``tests/``.

Kernel debugging (SURVEY §5.2 — the CUDA-sanitizer / launch-blocking role):

* ``HYPERION_DEBUG_BUILD=1`` loads ``_C_debug.so`` (``python -m hyperion.csrc.build --debug``:
  ``-O1 -g`` with the ``HYP_DASSERT`` device bounds checks) instead of ``_C.so``;
* ``HYPERION_KERNEL_CHECK=1`` wraps every native entry point: outside graph capture each call is
  followed by a device synchronize, so an asynchronous fault or launch error is reported AT the op
  that caused it (``RuntimeError: hyperion kernel check: <op> ...``); ``HYPERION_KERNEL_CHECK=nan``
  additionally scans the op's tensor outputs and names the first op that produced NaN/Inf.
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
STAT_SLOTS = 8  # hyp::kStatSlots: BN statistics sums are [STAT_SLOTS, 2, C] fp64 (csrc/hyp_kernels.h);
#                 checked against the loaded extension's STAT_SLOTS in _load()


def _load():
    global _MOD, _ERR, _TRIED
    if _TRIED:
        return _MOD
    _TRIED = True
    name = "hyperion._C_debug" if os.environ.get("HYPERION_DEBUG_BUILD") == "1" else "hyperion._C"
    try:
        _MOD = importlib.import_module(name)
    except BaseException as e:  # noqa: BLE001 - report any load failure
        _ERR = e
        _MOD = None
    if _MOD is not None and getattr(_MOD, "STAT_SLOTS", STAT_SLOTS) != STAT_SLOTS:
        raise RuntimeError(f"{name}: built with kStatSlots={_MOD.STAT_SLOTS}, Python expects {STAT_SLOTS}; rebuild")
    if _MOD is not None and os.environ.get("HYPERION_WS_DEPTH") and hasattr(_MOD, "ws_set_depth"):
        _MOD.ws_set_depth(int(os.environ["HYPERION_WS_DEPTH"]))  # weight-streaming k-steps in flight (A/B)
    if _MOD is not None and os.environ.get("HYPERION_CONV_PERSIST") and hasattr(_MOD, "conv_set_persist"):
        _MOD.conv_set_persist(int(os.environ["HYPERION_CONV_PERSIST"]))  # persistent fwd/dgrad convs (A/B)
    if _MOD is not None and os.environ.get("HYPERION_SPLITK_INKERNEL") and hasattr(_MOD, "gemm_set_splitk_inkernel"):
        _MOD.gemm_set_splitk_inkernel(int(os.environ["HYPERION_SPLITK_INKERNEL"]))  # 0: separate reduce (A/B)
    if _MOD is not None and os.environ.get("HYPERION_BN_GEOM") and hasattr(_MOD, "bn_set_geom"):
        b, it = (int(v) for v in os.environ["HYPERION_BN_GEOM"].split(","))  # "blocks,iters" (A/B)
        _MOD.bn_set_geom(b, it)
    if _MOD is not None and os.environ.get("HYPERION_CONV_GROUP") and hasattr(_MOD, "conv_set_group"):
        _MOD.conv_set_group(int(os.environ["HYPERION_CONV_GROUP"]))  # tile-order group sweep (A/B)
    if _MOD is not None and os.environ.get("HYPERION_ACT_COLSUM_WGS") and hasattr(_MOD, "colsum_set_act_wgs"):
        _MOD.colsum_set_act_wgs(int(os.environ["HYPERION_ACT_COLSUM_WGS"]))  # act_bwd_colsum grid (A/B)
    if _MOD is not None and os.environ.get("HYPERION_COLSUM_FIN_LANES") and hasattr(_MOD, "colsum_set_fin_lanes"):
        _MOD.colsum_set_fin_lanes(int(os.environ["HYPERION_COLSUM_FIN_LANES"]))  # final combine width (A/B)
    if _MOD is not None and os.environ.get("HYPERION_LN_WAVES") and hasattr(_MOD, "ln_set_waves"):
        _MOD.ln_set_waves(int(os.environ["HYPERION_LN_WAVES"]))  # LayerNorm grid sweep (A/B)
    if _MOD is not None and os.environ.get("HYPERION_ATTN_QSPLIT") and hasattr(_MOD, "attn_set_qsplit"):
        _MOD.attn_set_qsplit(int(os.environ["HYPERION_ATTN_QSPLIT"]))  # attention bwd query split (A/B)
    if _MOD is not None and os.environ.get("HYPERION_ATTN_FWD_NARROW") and hasattr(_MOD, "attn_set_fwd_narrow"):
        _MOD.attn_set_fwd_narrow(int(os.environ["HYPERION_ATTN_FWD_NARROW"]))  # 1-wave forward grid (A/B)
    mode = os.environ.get("HYPERION_KERNEL_CHECK", "")
    if _MOD is not None and mode:
        _MOD = CheckedModule(_MOD, nan=mode == "nan")
    return _MOD


class KernelCheckError(RuntimeError):
    pass


def _tensors(out):
    if isinstance(out, torch.Tensor):
        yield out
    elif isinstance(out, (list, tuple)):
        for o in out:
            yield from _tensors(o)


class CheckedModule:
    """Proxy of the extension whose functions synchronize (and optionally NaN-scan) after each call."""

    def __init__(self, mod, nan: bool = False):
        self._mod, self._nan = mod, nan
        self.__file__ = getattr(mod, "__file__", None)

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn
        nan = self._nan

        def wrapped(*args, **kw):
            out = fn(*args, **kw)
            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                try:
                    torch.cuda.synchronize()
                except RuntimeError as e:  # the asynchronous fault surfaces here, named
                    raise KernelCheckError(f"hyperion kernel check: {name} failed on the device: {e}") from e
                if nan:
                    for t in _tensors(out):
                        if t.is_floating_point() and t.numel() and not torch.isfinite(t).all():
                            raise KernelCheckError(f"hyperion kernel check: {name} produced NaN/Inf "
                                                   f"(output {tuple(t.shape)} {t.dtype})")
            return out

        return wrapped


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


# fp32 eager layers on the vendor ops (A/B: HYPERION_FP32_FUSED=1 keeps the fused autograd Functions).
# fp32 is outside the MFMA bf16/fp16 kernels: the fused Functions then only save an epilogue launch
# (bias+ReLU, dropout) and cost ~20-30 us of Python host time each per forward+backward — the fp32
# CustomTransformer row (512 tokens, launch-bound) ran 5.66 ms vs torch's 4.13 ms through them
# (profiles/r05/ct32_host_profile_*.txt).
PLAIN_FP32 = os.environ.get("HYPERION_FP32_FUSED", "0") != "1"


def plain_fp32(x: torch.Tensor) -> bool:
    """True when a linear / linear+activation on ``x`` should run as plain vendor ops (fp32 eager)."""
    return PLAIN_FP32 and x.dtype == torch.float32 and not torch.is_autocast_enabled(x.device.type)


class _InferCtx:
    """Stand-in ``ctx`` for calling an autograd Function's forward directly under ``no_grad``."""

    needs_input_grad = (False,) * 32

    def save_for_backward(self, *tensors):
        pass

    def mark_non_differentiable(self, *tensors):
        pass

    def mark_dirty(self, *tensors):
        pass

    def set_materialize_grads(self, value):
        pass


def apply_fn(fn, *args):
    """``fn.apply(*args)``, or — with grad mode off (eval / inference) — ``fn.forward`` on a stand-in
    ctx: the same kernels without the autograd-node bookkeeping, which costs ~10 us of host time per
    op and made the launch-bound fused inference of LM-768 slower than torch eager."""
    if torch.is_grad_enabled():
        return fn.apply(*args)
    return fn.forward(_InferCtx(), *args)


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


def rng_state(device: torch.device, increment: int = 8) -> torch.Tensor:
    """A graph-safe (seed, offset) record from torch's default generator for the counter-based
    dropout kernels (advances the generator like one torch dropout call)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return native().rng_state(idx, increment)


class ZeroArena:
    """Pre-zeroed fp64 workspace for the kernels' atomic accumulators (BN statistics sums).

    The BN kernels ADD per-channel sums into [2, C] fp64 buffers with f64 atomics, so every
    buffer must be zero before its producer runs.  A fresh ``torch.zeros`` per BN layer would be one
    fill launch each (~100 per ResNet-50 step); instead a model opens ``zero_scope`` around its
    forward and every BN call takes a slice of ONE buffer zeroed by a single fill (the forward's
    and, reserved at forward time, the backward's sums).  The first call under a key learns the
    size; later calls preallocate it.  Without an open scope (or past the learnt size), ``take``
    returns a fresh zeroed tensor — always correct, just one fill more.  Slices keep the buffer
    alive, so a later scope never recycles memory an unfinished backward still reads.
    """

    ALIGN = 32  # doubles (256 B): every slice starts on its own 256-byte run

    def __init__(self, buf: Optional[torch.Tensor]):
        self.buf = buf
        self.off = 0
        self.used = 0

    def take(self, n: int, device) -> torch.Tensor:
        need = -(-n // self.ALIGN) * self.ALIGN
        self.used += need
        if self.buf is not None and self.buf.device == torch.device(device) and self.off + need <= self.buf.numel():
            t = self.buf[self.off:self.off + n]
            self.off += need
            return t
        return torch.zeros(n, device=device, dtype=torch.float64)


_ARENAS: list = []


class zero_scope:
    """``with zero_scope(owner, key, device):`` — one zero-fill for every accumulator taken inside
    (nested scopes reuse the outermost).  ``owner`` keeps the learnt size per ``key``."""

    def __init__(self, owner, key: str, device):
        self.owner, self.key, self.device = owner, key, torch.device(device)
        self.arena = None

    def __enter__(self):
        if _ARENAS or self.device.type != "cuda":
            return self
        sizes = self.owner.__dict__.setdefault("_zero_arena_sizes", {})
        # a key not seen yet (a graph stage captured after warm-up ran the whole forward) borrows
        # the largest learnt size: one fill of a slightly larger buffer instead of one per layer
        n = sizes.get(self.key, 0) or max(sizes.values(), default=0)
        self.arena = ZeroArena(torch.zeros(n, device=self.device, dtype=torch.float64) if n else None)
        _ARENAS.append(self.arena)
        return self

    def __exit__(self, *exc):
        if self.arena is not None:
            _ARENAS.pop()
            sizes = self.owner.__dict__["_zero_arena_sizes"]
            sizes[self.key] = max(sizes.get(self.key, 0), self.arena.used)
        return False


def zeroed(n: int, device) -> torch.Tensor:
    """A zeroed fp64 [n] accumulator: a slice of the open ``zero_scope`` arena, else fresh."""
    if _ARENAS:
        return _ARENAS[-1].take(n, device)
    return torch.zeros(n, device=device, dtype=torch.float64)
