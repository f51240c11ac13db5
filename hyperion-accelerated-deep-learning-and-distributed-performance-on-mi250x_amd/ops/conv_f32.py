"""fp32 convolution on the fp32-input MFMA GEMM (``csrc/kernels/gemm_f32.hip``) — no MIOpen.

Reference: the reference-methodology model benchmarks run fp32 (``Phase 1/baseline_performance.ipynb:
252-358``: ResNet-50, the fallback CNN; ``02_development/compilation_optimization.py:47-51`` ``--dtype
fp32``), every convolution a MIOpen fp32 kernel (SURVEY C6 / C32, §2.4 "Convolution").  The bf16 /
fp16 implicit-GEMM kernels (``conv_igemm.hip``) are built around the 16-bit MFMA fragments; fp32
gets its own path, designed for what fp32 costs on gfx950:

* the fp32 MFMA (v_mfma_f32_32x32x2_f32) spends 64 cycles per 32x32x2 step, so a convolution is
  MFMA-bound long before the im2col bytes matter: forward = NHWC im2col (one bandwidth pass,
  ``im2col_f32``) + ONE fp32 GEMM ``cols · Wᵀ`` with the bias in its epilogue; a 1x1 / stride-1
  convolution reads the channels-last activation directly (no im2col);
* backward = the weight gradient ``dyᵀ · cols`` (both operands read transposed in-kernel, split-K
  over the output pixels, deterministic slab reduce) and the data gradient ``dy · W`` (the filter
  read transposed) followed by ``col2im_f32`` — a per-input gather over the taps (no atomics);
* the im2col matrix of the forward is kept for the weight gradient (288 GB of HBM: ~1.5 GB for a
  ResNet-50 batch of 32) instead of being rebuilt.

Exact fp32 products and fp32 accumulation (gfx950 has no TF32-like MFMA) — the numerics of
``F.conv2d`` in fp32 up to summation order.  ``HYPERION_CONV_F32=0`` restores the vendor kernels.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native

ENABLED = os.environ.get("HYPERION_CONV_F32", "1") == "1"
# Launch plans: the kernel's cost model picks (tile shape, split-K) for a shape it has not seen; with
# tuning on, the first eager call of each (layout, M, N, K) times the model's neighbourhood on the
# call's own operands and caches the fastest ("measure, don't guess"; the bf16 GEMM's autotuner).
TUNE = os.environ.get("HYPERION_F32_TUNE", "1") == "1"
_PLAN: Dict[tuple, Tuple[int, int]] = {}
_SPLITS = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128)


def _tune(C, a, b, a_tr: bool, b_tr: bool, K: int) -> Tuple[int, int]:
    from .gemm import _time

    nk = (K + 31) // 32
    best, plan = _time(lambda: C.gemm_f32(a, b, a_tr=a_tr, b_tr=b_tr), reps=3), (-1, -1)
    for shape in (0, 1, 2):  # 3 / 4 (one workgroup per CU) measured slower everywhere
        for sp in _SPLITS:
            if sp > 1 and nk // sp < 2:
                break
            t = _time(lambda: C.gemm_f32(a, b, a_tr=a_tr, b_tr=b_tr, shape=shape, splits=sp), reps=3)
            if t < best * 0.97:
                best, plan = t, (shape, sp)
    return plan


def gemm(a: torch.Tensor, b: torch.Tensor, a_tr: bool = False, b_tr: bool = False, **kw) -> torch.Tensor:
    """``C.gemm_f32`` with the per-shape launch plan (tuned on first eager use when TUNE)."""
    C = _native.native()
    M, K = (a.shape[1], a.shape[0]) if a_tr else (a.shape[0], a.shape[1])
    N = b.shape[1] if b_tr else b.shape[0]
    key = (a_tr, b_tr, M, N, K)
    plan = _PLAN.get(key)
    if plan is None:
        plan = (-1, -1)
        if TUNE and not torch.cuda.is_current_stream_capturing():
            plan = _tune(C, a, b, a_tr, b_tr, K)
            _PLAN[key] = plan
    return C.gemm_f32(a, b, a_tr=a_tr, b_tr=b_tr, shape=plan[0], splits=plan[1], **kw)


def f32_conv_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    w = conv.weight
    return (ENABLED and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and w.dtype == torch.float32
            and conv.groups == 1 and tuple(conv.dilation) == (1, 1) and isinstance(conv.padding, tuple)
            and conv.padding_mode == "zeros" and w.shape[0] % 4 == 0
            and not torch.is_autocast_enabled(x.device.type)
            and _native.use_native(x, op="conv"))


def _wmat(w: torch.Tensor, kp: int) -> torch.Tensor:
    """[Cout, Cin, R, S] -> [Cout, Kp] with column (r*S + s)*Cin + c (the im2col order), zero pad
    columns past R*S*Cin.  A channels-last weight is a free view."""
    co = w.shape[0]
    m = w.permute(0, 2, 3, 1).reshape(co, -1)
    if m.shape[1] != kp:
        m = F.pad(m, (0, kp - m.shape[1]))
    return m if m.is_contiguous() else m.contiguous()


class _Conv2dF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride: Tuple[int, int], padding: Tuple[int, int]):
        C = _native.native()
        if not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        nb, cin, h, wd = x.shape
        co, _, r, s = w.shape
        (sh, sw), (ph, pw) = stride, padding
        ho, wo = (h + 2 * ph - r) // sh + 1, (wd + 2 * pw - s) // sw + 1
        kp = (r * s * cin + 3) // 4 * 4
        wm = _wmat(w, kp)
        direct = r == 1 and s == 1 and sh == 1 and sw == 1 and ph == 0 and pw == 0 and cin % 4 == 0
        cols = x.permute(0, 2, 3, 1).reshape(nb * h * wd, cin) if direct else C.im2col_f32(x, r, s, sh, sw, ph, pw, kp)
        # the output is allocated channels-last and written through a [M, Cout] view, so the
        # Function returns a base tensor (callers may apply an in-place ReLU to it)
        y = torch.empty((nb, co, ho, wo), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        gemm(cols, wm, bias=b, out=y.permute(0, 2, 3, 1).view(nb * ho * wo, co))
        ctx.save_for_backward(cols if ctx.needs_input_grad[1] else None, wm if ctx.needs_input_grad[0] else None)
        ctx.geom = (nb, cin, h, wd, co, r, s, sh, sw, ph, pw, ho, wo, kp, direct, b is not None)
        _native.count("conv_f32")
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _native.native()
        cols, wm = ctx.saved_tensors
        nb, cin, h, wd, co, r, s, sh, sw, ph, pw, ho, wo, kp, direct, has_b = ctx.geom
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dy2 = dy.permute(0, 2, 3, 1).reshape(nb * ho * wo, co)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dcols = gemm(dy2, wm, b_tr=True)  # [M, Kp] = dy · W
            if direct:
                dx = dcols.view(nb, h, wd, cin).permute(0, 3, 1, 2)
            else:
                dx = C.col2im_f32(dcols, nb, cin, h, wd, r, s, sh, sw, ph, pw)
        if ctx.needs_input_grad[1]:
            dwm = gemm(dy2, cols, a_tr=True, b_tr=True)  # [Cout, Kp] = dyᵀ · cols
            dw = dwm[:, : r * s * cin].reshape(co, r, s, cin).permute(0, 3, 1, 2)
        if has_b and ctx.needs_input_grad[2]:
            db = dy2.sum(0)
        return dx, dw, db, None, None


# Per-convolution routing: the native path and the vendor convolution are timed (forward + both
# gradients, on operands of the call's shape) on the first eager call of each geometry and the faster
# runs from then on — the fp32 MFMA GEMM wins some ResNet shapes and loses others to MIOpen
# (profiles/r06/fp32_conv_routes_resnet50.txt), so per-layer routing beats either side alone.  ROUTE=native
# forces the native path (tests, traces), ROUTE=vendor the vendor one.
ROUTE = os.environ.get("HYPERION_CONV_F32_ROUTE", "auto")
_ROUTE: Dict[tuple, bool] = {}
ROUTE_MS: Dict[tuple, Tuple[float, float]] = {}  # key -> (native, vendor) ms per fwd + bwd (records)


def _native_faster(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    if ROUTE != "auto":
        return ROUTE == "native"
    w, b = conv.weight, conv.bias
    # geometry only: a no-grad call (an inference loop after training warm-up) reuses the decision
    key = (tuple(x.shape), tuple(w.shape), tuple(conv.stride), tuple(conv.padding), b is not None)
    c = _ROUTE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return True
        from .gemm import _time

        xt = torch.randn(x.shape, device=x.device).contiguous(memory_format=torch.channels_last)
        xt.requires_grad_(x.requires_grad)
        wt = w.detach().clone().requires_grad_(w.requires_grad)
        bt = b.detach().clone().requires_grad_(b.requires_grad) if b is not None else None
        ins = [t for t in (xt, wt, bt) if t is not None and t.requires_grad]

        def run(native):
            with torch.enable_grad():
                y = (_Conv2dF32Fn.apply(xt, wt, bt, tuple(conv.stride), tuple(conv.padding)) if native
                     else F.conv2d(xt, wt, bt, conv.stride, conv.padding))
                if ins:
                    torch.autograd.grad(y, ins, torch.ones_like(y))

        run(True)
        run(False)
        tn, tv = _time(lambda: run(True), reps=3) / 3, _time(lambda: run(False), reps=3) / 3
        c = tn < tv
        _ROUTE[key] = c
        ROUTE_MS[key] = (tn, tv)
    return c


def conv2d_f32(x: torch.Tensor, conv: nn.Conv2d) -> Optional[torch.Tensor]:
    """``conv(x)`` for an fp32 ``nn.Conv2d`` on the native fp32 path (channels-last output), or None
    when the vendor convolution measured faster for this geometry (the caller runs it)."""
    if not _native_faster(x, conv):
        return None
    return _native.apply_fn(_Conv2dF32Fn, x, conv.weight, conv.bias, tuple(conv.stride), tuple(conv.padding))


class Conv2d(nn.Conv2d):
    """Drop-in ``nn.Conv2d`` (same parameters and state-dict keys) whose fp32 GPU forward runs on
    the native fp32 path; bf16 / fp16 / CPU calls are ``nn.Conv2d``'s own."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        if f32_conv_ok(x, self):
            y = conv2d_f32(x, self)
            if y is not None:
                return y
        return super().forward(x)


def conv2d_f32_reference(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], stride, padding) -> torch.Tensor:
    """The oracle of the GPU tests (fp64 on the CPU)."""
    return F.conv2d(x.double().cpu(), w.double().cpu(), None if b is None else b.double().cpu(), stride, padding)


# ---- inference: conv -> BN(running stats) -> (+ residual) -> (ReLU) with the BN folded -------------------
# (the filter rows scaled by γ/σ, the shift as the GEMM's bias, ReLU in its epilogue when there is no
# residual): one im2col + one GEMM per layer instead of a conv, a BN pass and a ReLU pass.  Routed
# per geometry against the vendor conv + BN the same way as training (forward timing only).
_EVAL_ROUTE: Dict[tuple, bool] = {}


def _folded(conv: nn.Conv2d, sc: torch.Tensor, sh: torch.Tensor, kp: int):
    w = conv.weight
    key = (w.data_ptr(), w._version, sc.data_ptr(), sh.data_ptr(),
           None if conv.bias is None else (conv.bias.data_ptr(), conv.bias._version))
    cache = conv.__dict__.get("_hyp_f32_folded")
    if cache is not None and cache[0] == key:
        return cache[1], cache[2]
    with torch.no_grad():
        wm = _wmat(w * sc.view(-1, 1, 1, 1), kp)
        b = sh + conv.bias.float() * sc if conv.bias is not None else sh
        b = b.contiguous()
    conv.__dict__["_hyp_f32_folded"] = (key, wm, b)
    return wm, b


def _eval_native(conv, x, residual, act, sc, sh):
    C = _native.native()
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    nb, cin, h, wd = x.shape
    co, _, r, s = conv.weight.shape
    (sh_, sw), (ph, pw) = tuple(conv.stride), tuple(conv.padding)
    ho, wo = (h + 2 * ph - r) // sh_ + 1, (wd + 2 * pw - s) // sw + 1
    kp = (r * s * cin + 3) // 4 * 4
    wm, bias = _folded(conv, sc, sh, kp)
    direct = r == 1 and s == 1 and sh_ == 1 and sw == 1 and ph == 0 and pw == 0 and cin % 4 == 0
    cols = x.permute(0, 2, 3, 1).reshape(nb * h * wd, cin) if direct else C.im2col_f32(x, r, s, sh_, sw, ph, pw, kp)
    y = torch.empty((nb, co, ho, wo), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    gemm(cols, wm, bias=bias, relu=bool(act) and residual is None, out=y.permute(0, 2, 3, 1).view(nb * ho * wo, co))
    if residual is not None:
        y.add_(residual)
        if act:
            y.relu_()
    return y


def conv_bn_eval_f32(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor, residual: Optional[torch.Tensor],
                     sc: torch.Tensor, sh: torch.Tensor) -> Optional[torch.Tensor]:
    """fp32 inference conv + BN (+ residual) (+ ReLU) with the BN folded (None: the caller's path)."""
    if not f32_conv_ok(x, conv) or torch.is_grad_enabled():
        return None
    act = bool(getattr(bn, "act", False))
    if residual is not None and (residual.dtype != x.dtype or residual.shape[0] != x.shape[0]):
        return None
    key = (tuple(x.shape), tuple(conv.weight.shape), tuple(conv.stride), tuple(conv.padding), residual is not None)
    c = _EVAL_ROUTE.get(key) if ROUTE == "auto" else ROUTE == "native"
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            c = True
        else:
            from .gemm import _time

            def vendor():
                y = F.batch_norm(F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding), bn.running_mean,
                                 bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
                if residual is not None:
                    y = y + residual
                return F.relu(y) if act else y

            _eval_native(conv, x, residual, act, sc, sh)
            vendor()
            c = _time(lambda: _eval_native(conv, x, residual, act, sc, sh), reps=3) < _time(vendor, reps=3)
            _EVAL_ROUTE[key] = c
    if not c:
        return None
    _native.count("conv_bn_eval_f32")
    return _eval_native(conv, x, residual, act, sc, sh)
