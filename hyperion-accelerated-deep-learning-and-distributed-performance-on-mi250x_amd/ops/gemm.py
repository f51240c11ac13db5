"""Transformer-size GEMMs on the deep-pipelined MFMA kernel (``csrc/kernels/gemm_tiles.hip``).

Reference: every ``nn.Linear`` / ``nn.TransformerEncoderLayer`` / ViT MLP GEMM of the reference
runs on hipBLASLt (``02_development/distributed_utils.py:75-88``, ``Phase 1/baseline_performance.ipynb``
cells 238-249; SURVEY §2.4 "GEMM").  Here the three GEMMs of a linear layer are one kernel family
with no transposed copies:

* ``mm_nt(x, w)``  forward ``x Wᵀ`` (+ bias, ReLU/GELU with the pre-activation kept, + residual);
* ``mm_nn(dy, w)`` data gradient ``dy W`` (W read transposed in-kernel, ds_read_b64_tr_b16);
* ``mm_tn(dy, x)`` weight gradient ``dyᵀ x`` (both operands read transposed), optionally
  accumulated (``beta = 1``) into an fp32 buffer.

Routing ("measure, don't guess"): the first eager call of a (layout, M, N, K, epilogue) shape
times the vendor GEMM and the tiled kernel at every (tile, split-K) candidate on the call's own
operands (a few repetitions each) and caches the winner — the tiled kernel's (tile, splits) or
the vendor; under hipGraph capture an unseen shape takes the tiled kernel's static plan.  ``HYPERION_GEMM=vendor|native|auto`` (default
auto) forces either side — the numerics tests and A/B runs use it.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from . import _native

_MODE = os.environ.get("HYPERION_GEMM", "auto")
_CHOICE: Dict[Tuple, Optional[Tuple[int, int]]] = {}  # shape key -> (tile, splits) or None (vendor)
ACTS = {None: 0, "none": 0, "relu": 1, "gelu": 2, "gelu_tanh": 3}


def set_mode(mode: str) -> None:
    """'auto' (timed per shape), 'native' (always the tiled kernel) or 'vendor' (hipBLASLt)."""
    global _MODE
    assert mode in ("auto", "native", "vendor")
    _MODE = mode
    _CHOICE.clear()


def choices() -> Dict[Tuple, Optional[Tuple[int, int]]]:
    return dict(_CHOICE)


def _ok(*ts: torch.Tensor) -> bool:
    t0 = ts[0]
    return (_MODE != "vendor" and t0.is_cuda and t0.dtype in (torch.bfloat16, torch.float16)
            and all(t.dtype == t0.dtype and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0
                    and t.data_ptr() % 16 == 0 for t in ts)
            and _native.use_native(t0, op="gemm"))


def _time(fn, reps: int = 5) -> float:
    """Device time of one call: the calls are queued behind a spin kernel (torch.cuda._sleep) so the
    events bracket GPU work only — host launch overhead (comparable to these 10-50 us GEMMs) must
    not decide the choice, because the training step replays them from a hipGraph."""
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)  # ~1 ms of queue ahead of the timed calls
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


# (BM, BN) of the tiled kernel's tiles (gemm_tiles.hip kTiles; 3 = the ragged-shape 128x128;
# 8-11 = the ping-pong kernel gemm_pp_k)
TILES = {0: (256, 256), 1: (256, 128), 2: (128, 128), 4: (64, 64), 5: (128, 64), 6: (64, 128), 7: (192, 128),
         8: (256, 256), 9: (256, 128), 10: (128, 256), 11: (128, 128), 12: (256, 256)}


def _candidates(K: int, M: int = 1 << 30, N: int = 1 << 30, a_tr: bool = False, b_tr: bool = False):
    """(tile, splits) pairs worth timing: tiles the layout can stage (a transposed operand needs a
    128-multiple tile side) and that fit the output, split-K slices >= 256 deep."""
    for t, (bm, bn) in TILES.items():
        if (a_tr and bm % 128) or (b_tr and bn % 128) or bm > M or bn > N:
            continue
        for sp in (1, 2, 3, 4, 6, 8, 12, 16):
            if sp == 1 or K // sp >= 256:
                yield (t, sp)


def _pick(key: Tuple, K: int, native_fn, vendor_fn, M: int = 1 << 30, N: int = 1 << 30, a_tr: bool = False,
          b_tr: bool = False) -> Optional[Tuple[int, int]]:
    """(tile, splits) for the tiled kernel, (-1, -1) = its static plan, or None = vendor."""
    if _MODE == "native":
        return _CHOICE.get(key, (-1, -1)) or (-1, -1)
    if key in _CHOICE:
        return _CHOICE[key]
    if torch.cuda.is_current_stream_capturing():
        return (-1, -1)  # no timing under capture: static plan
    best, bt = _time(vendor_fn), None
    for c in _candidates(K, M, N, a_tr, b_tr):
        try:
            tc = _time(lambda: native_fn(*c))
        except RuntimeError:  # a (tile, layout) the kernel refuses
            continue
        if tc < best:
            best, bt = tc, c
    _CHOICE[key] = bt
    return bt


def mm_nt(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act: Optional[str] = None,
          aux: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None, dropout_p: float = 0.0,
          rng: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """``act(x Wᵀ + bias) (+ residual)`` with ``aux`` = pre-activation, or None when the vendor path
    should run (the caller keeps its own fallback).  ``dropout_p`` (with ``act``): the output is
    ``dropout(act(...))`` with the mask of the ``rng`` record (the FFN's inner dropout in the epilogue)."""
    if not _ok(x, w) or x.shape[1] % 8 or w.shape[0] % 4:
        return None
    if residual is not None and (residual.dtype != x.dtype or residual.stride(1) != 1 or residual.stride(0) % 4):
        return None
    if bias is not None and (not bias.is_contiguous() or bias.data_ptr() % 16 or bias.dtype not in
                             (torch.float32, torch.bfloat16, torch.float16)):
        return None
    C = _native.native()
    a = ACTS[act]
    key = ("nt", x.shape[0], w.shape[0], x.shape[1], a, bias is not None, residual is not None, dropout_p > 0)

    def nat(tile=-1, splits=-1):
        return C.gemm(x, w, bias=bias, act=a, aux=aux, residual=residual, tile=tile, splits=splits,
                      drop_p=dropout_p, rng=rng)

    def ven():
        y = torch.addmm(bias.to(x.dtype), x, w.t()) if bias is not None else x @ w.t()
        if a == 2:  # what the vendor fallback of linear_act runs: GELU + dropout in one native pass
            h = C.dropout(y, dropout_p, rng, act=2)
            return h + residual if residual is not None else h  # (no "+ 0": an extra full-size add kernel)
        if a == 1:
            y = torch.relu(y)
        elif a == 3:
            y = torch.nn.functional.gelu(y, approximate="tanh")
        if dropout_p > 0:
            y = C.dropout(y, dropout_p, rng)
        return y + residual if residual is not None else y

    c = _pick(key, x.shape[1], nat, ven, x.shape[0], w.shape[0])
    if c is None:
        return None
    _native.count("gemm_nt")
    return nat(*c)


def mm_nn(dy: torch.Tensor, w: torch.Tensor, residual: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """``dy W`` (dy [M, N], W [N, K]) ``(+ residual)`` (added in the epilogue: a data gradient that
    also receives a residual branch's gradient) or None (vendor)."""
    if not _ok(dy, w) or w.shape[1] % 4 or dy.shape[1] % 8:
        return None
    if residual is not None and (residual.dtype != dy.dtype or residual.stride(1) != 1 or residual.stride(0) % 4):
        return None
    C = _native.native()
    key = ("nn", dy.shape[0], w.shape[1], dy.shape[1]) + (("res",) if residual is not None else ())
    ven = (lambda: dy @ w) if residual is None else (lambda: torch.addmm(residual, dy, w))
    c = _pick(key, dy.shape[1], lambda t=-1, sp=-1: C.gemm(dy, w, b_tr=True, residual=residual, tile=t, splits=sp),
              ven, dy.shape[0], w.shape[1], b_tr=True)
    if c is None:
        return None
    _native.count("gemm_nn")
    return C.gemm(dy, w, b_tr=True, residual=residual, tile=c[0], splits=c[1])


def mm_tn(dy: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None, beta: float = 0.0,
          out_dtype: Optional[torch.dtype] = None) -> Optional[torch.Tensor]:
    """``dyᵀ x`` (dy [T, N], x [T, K] -> [N, K]); ``out``/``beta`` accumulate, or None (vendor)."""
    if not _ok(dy, x) or dy.shape[1] % 8 or x.shape[1] % 8 or dy.shape[0] % 8:
        return None
    C = _native.native()
    key = ("tn", dy.shape[1], x.shape[1], dy.shape[0])
    odt = out.dtype if out is not None else (out_dtype or dy.dtype)

    def ven():
        return (dy.t() @ x).to(odt)

    c = _pick(key, dy.shape[0], lambda t=-1, sp=-1: C.gemm(dy, x, a_tr=True, b_tr=True, out_dtype=odt, tile=t,
                                                           splits=sp), ven, dy.shape[1], x.shape[1], True, True)
    if c is None:
        return None
    _native.count("gemm_tn")
    return C.gemm(dy, x, a_tr=True, b_tr=True, out_dtype=None if out is not None else odt, out=out, beta=beta,
                  tile=c[0], splits=c[1])


# ---- LM head (V = 50257 classes: N % 4 != 0) ------------------------------------------------------
def lm_head_logits(x: torch.Tensor, w: torch.Tensor, zb: torch.Tensor) -> bool:
    """Logits ``x Wᵀ`` into ``zb[:, :V]`` (``zb`` [N, ceil8(V)], 16-byte aligned rows) on the native
    GEMM: classes [0, floor8(V)) on the tiled kernel, the last V % 8 classes and the row padding as
    one small launch whose weight rows past V read as zeros (the padding columns come out 0, so
    the backward GEMMs that reduce over classes read finite zeros there).  False: the caller runs
    the vendor GEMM (the autotuner found it faster, or the operands do not qualify)."""
    V, Vp = w.shape[0], zb.shape[1]
    Vm = V // 8 * 8
    if not _ok(x, w) or x.shape[1] % 8 or Vm < 256 or Vp % 8 or Vp < V:
        return False
    C = _native.native()
    key = ("lm_head", x.shape[0], V, x.shape[1])

    def nat(tile=-1, splits=-1):
        C.gemm(x, w[:Vm], out=zb[:, :Vm], tile=tile, splits=splits)
        if Vp > Vm:
            C.gemm(x, w[Vm:], out=zb[:, Vm:], n_out=Vp - Vm)
        return zb

    def ven():
        return torch.mm(x, w.t(), out=zb[:, :V])

    c = _pick(key, x.shape[1], nat, ven, x.shape[0], Vm)
    if c is None:
        return False
    _native.count("gemm_lm_head")
    nat(*c)
    return True


def lm_head_dx(zb: torch.Tensor, w: torch.Tensor) -> Optional[torch.Tensor]:
    """``dz W`` reducing over the V classes of ``zb[:, :V]`` (its padding columns must be finite:
    lm_head_logits writes zeros there) — one launch: the reduction's ragged end (V % 32) is staged
    per lane with the weight rows past V read as zeros.  None = vendor."""
    V = w.shape[0]
    z = zb[:, :V]
    if not _ok(zb, w) or w.shape[1] % 8:
        return None
    C = _native.native()
    key = ("lm_head_dx", zb.shape[0], w.shape[1], V)
    c = _pick(key, V, lambda t=-1, sp=-1: C.gemm(z, w, b_tr=True, tile=t, splits=sp),
              lambda: torch.mm(z, w), zb.shape[0], w.shape[1], b_tr=True)
    if c is None:
        return None
    _native.count("gemm_lm_head_dx")
    return C.gemm(z, w, b_tr=True, tile=c[0], splits=c[1])
