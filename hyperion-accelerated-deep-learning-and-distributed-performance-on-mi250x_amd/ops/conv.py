"""Convolution + BatchNorm (+ residual) (+ ReLU) on the gfx950 implicit-GEMM kernel.

Reference: every ResNet ``conv → bn → relu`` (and ``conv → bn → += identity → relu``) ran as a
MIOpen convolution plus a MIOpen BN (statistics pass, normalize pass) plus separate ReLU / add
kernels (``baseline_performance.ipynb:203-205``, torchvision ResNet-18 in ``distributed_utils.py:229``;
SURVEY §2.4 "Convolution + BatchNorm + ReLU", hard part #1 in §7.4).

``conv_bn_act(conv, bn, x, residual)`` (training mode, bf16/f16 channels-last):

* forward  — ``csrc/kernels/conv_igemm.hip`` computes the convolution on MFMA AND adds the
  per-channel Σy, Σy² of its (rounded) outputs into a zeroed accumulator in the epilogue (float
  atomics); BN then runs ONE apply launch that finalizes the statistics inline, with the residual
  add and ReLU folded in (``bn_act.hip``).  No separate statistics read, no finalize launch.
  ``defer=True`` (a ``conv → BN → ReLU`` whose output feeds a stride-1 "same"-padded conv, i.e.
  every bottleneck's conv1 → conv2 → conv3 chain): no apply launch at all — the CONSUMING conv
  reads the raw conv output and applies BN + ReLU to its A operand as it reads it (the kernel's
  XF mode), storing the activation the backward needs as a side output (SURVEY §2.4 "BN-apply
  + ReLU stage in the next conv's prologue").  Opt-in (``HYPERION_CONV_XF=1x1|all``): measured
  on MI355X it does not beat the apply pass — the latency-bound conv kernels pay the transform on
  every K step's critical path, a 3x3 once per tap (README "Measured non-wins", profiles/r04/xf).
* backward — the fused BN/ReLU/residual backward (``bn_act.hip``) produces dconv; the data
  gradient of a stride-1 convolution is the same implicit-GEMM kernel in DGRAD mode (the forward
  filter read flipped and channel-transposed through ds_read_b64_tr_b16, no filter copy); a
  stride-2 RxS data gradient runs as its 4 output-phase sub-convolutions in ONE DGRAD launch; weight
  gradients run on ``conv_wgrad.hip`` (split-K MFMA over the output pixels); a 1x1 strided data
  gradient is the same DGRAD GEMM on the output grid plus one scatter(+add) pass; anything else
  uses the vendor kernels (``aten.convolution_backward``).

The RGB stem (7x7/s2/p3, C <= 4) is rewritten as space-to-depth + a stride-1 R=4 conv whose
64-element reduction runs span 4 adjacent 16-channel pixels (``stem.hip``), on the same kernels.  Anything else
outside the kernel's envelope (fp32, other C % 64 != 0 convs, groups, dilation, eval mode) falls
back to ``bn(conv(x), residual)`` — the same math.
"""
from __future__ import annotations

import os
import weakref
from typing import Optional

import torch
import torch.nn as nn

from . import _native
from . import streams as _streams


def _native_conv_ok(x: torch.Tensor, conv: nn.Conv2d, w: Optional[torch.Tensor] = None,
                    wdt: Optional[torch.dtype] = None) -> bool:
    """``wdt``: the dtype the weight will have at the call (autocast casts it), default its own."""
    w = conv.weight if w is None else w
    return (
        x.is_cuda
        and x.dim() == 4
        and x.dtype in (torch.bfloat16, torch.float16)
        and (w.dtype if wdt is None else wdt) == x.dtype
        and conv.groups == 1
        and tuple(conv.dilation) == (1, 1)
        and conv.bias is None
        and isinstance(conv.padding, tuple)
        and x.shape[1] % 64 == 0
        and w.shape[0] % 8 == 0
        and x.is_contiguous(memory_format=torch.channels_last)
        and w.is_contiguous(memory_format=torch.channels_last)
    )


# Tuned launch plans (the MIOpen find-db role): configs/conv_plans_mi355x.json, written by
# scripts/conv_tune.py on MI355X — per GEMM shape the fastest (tile, split-K, LDS ring depth) of
# the forward (+ BN statistics) and of the data gradient with the BN-backward epilogue; shapes not
# in the table use the kernels' own heuristics.  HYPERION_CONV_PLANS=<path> | off.
_PLANS: Optional[dict] = None


def _plan(op: str, M: int, K: int, C: int, R: int, S: int, stride: int):
    global _PLANS
    if _PLANS is None:
        _PLANS = {}
        path = os.environ.get("HYPERION_CONV_PLANS", "")
        if path != "off":
            if not path:
                path = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                    "configs", "conv_plans_mi355x.json")
            try:
                import json

                with open(path) as f:
                    for pl in json.load(f).get("plans", []):
                        key = (pl["op"], pl["M"], pl["K"], pl["C"], pl["R"], pl["S"], pl["stride"])
                        _PLANS[key] = (int(pl["bm"]), int(pl["bn"]), int(pl["splits"]), int(pl["stages"]),
                                       int(pl.get("order", -1)))
            except (OSError, ValueError, KeyError):
                _PLANS = {}
    return _PLANS.get((op, M, K, C, R, S, stride))


FUSE_BN_BACKWARD = True  # dgrad epilogue computes the producing BN layer's backward reduce (A/B switch)
# Producer kinds that take the epilogue (mode 0: BN without ReLU, 1: BN+ReLU, 2: BN+residual+ReLU).
# Mode 2 saves a 3-tensor reduce pass, the dx pass's y read and its dres write; modes 0/1 save only
# a 2-tensor reduce, about what the epilogue's extra x read costs the dgrad's store phase
# (scripts/bnb_tiles.py).  ResNet-50 bench on MI355X (scripts/gpu_ab_bnb.sh): none 5.73 ms,
# {2} 5.60, {1,2} 5.58, {0,1,2} 5.60.
FUSE_BN_MODES = {int(m) for m in os.environ.get("HYPERION_BNB_MODES", "1,2").split(",") if m.strip()}


class BNGradLink:
    """Hands the BatchNorm-backward reduction of a fused conv→BN(→+res)(→ReLU) layer (the
    PRODUCER) to the data gradient of the conv that consumes its output.

    The consumer's stride-1 dgrad kernel (``conv_igemm.hip`` BNB epilogue) then stores
    dz = dX·ReLU-mask instead of dX and adds Σdz, Σdz·x into the producer's zeroed sums, so the
    producer's backward is ONE dx pass (``bn_bwd_dx``) instead of a reduce pass + a dx pass, and
    its residual gradient is dz itself (no extra write).  Masking is idempotent, so handing dz to
    autograd is safe; the producer takes the fast path only when the gradient it receives IS that
    dz object (any other contribution summed by autograd, or an epilogue that never ran, sends it
    down the full path with fresh sums).  Each backward consumes the link once (``used``): a
    second backward over a retained graph takes the full path."""

    # no reference to the producer's OUTPUT here (it would be a ctx -> output -> grad_fn cycle):
    # the mode-2 mask source is the consumer's own saved input, which is that output
    __slots__ = ("yc", "bn_w", "bn_b", "mean", "invstd", "mode", "sums", "dz", "used")

    def __init__(self, yc, bn_w, bn_b, mean, invstd, mode, sums):
        self.yc, self.bn_w, self.bn_b = yc, bn_w, bn_b
        self.mean, self.invstd, self.mode, self.sums = mean, invstd, mode, sums
        self.dz = None
        self.used = False


# The layer's weight gradient in the data gradient's launch (csrc/kernels/conv_dual.hip): both read
# dY, neither reads the other — one launch per layer instead of two, and the two gradients' latency-
# bound workgroups overlap (skipping every weight gradient outright: 4.79 -> 3.81 ms per ResNet-50
# step, profiles/r05).  HYPERION_CONV_DUAL: "0" off (separate launches), "1" the two gradients'
# workgroups interleaved, "2" data-gradient workgroups first (default).  Same box, ResNet-50 step:
# separate 4.79 ms, interleaved 4.83-4.87 (other box), data gradient first 4.67 (profiles/r05/dual_ab.txt).
_DUAL = os.environ.get("HYPERION_CONV_DUAL", "2")


class WgradRequest:
    """The weight gradient ``_dgrad`` may compute in its own launch: the conv's input ``x`` and
    geometry; ``dw`` is set when it did (else the caller runs :func:`_wgrad`)."""

    __slots__ = ("x", "R", "S", "stride", "padding", "w_param", "dw")

    def __init__(self, x, w, stride, padding, w_param):
        self.x, self.R, self.S = x, w.shape[2], w.shape[3]
        self.stride, self.padding, self.w_param = tuple(stride), tuple(padding), w_param
        self.dw = None


def _wgrad_native_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    P, Q = dy.shape[2], dy.shape[3]
    return (x.shape[1] % 64 == 0 and dy.shape[1] % 8 == 0 and P * Q < (1 << 14) and dy.shape[0] * P * Q < (1 << 22)
            and _native.use_native(x, op="wgrad"))


def wgrad_request(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride, padding,
                  w_param: Optional[torch.Tensor] = None) -> Optional[WgradRequest]:
    """A request for :func:`_dgrad` when the fused launch applies (bf16 channels-last operands of one
    dtype, the native weight-gradient envelope), else None."""
    if WGRAD_FUSE != "dgrad" or _DUAL == "0" or _streams.enabled():
        return None
    if not (dy.dtype == torch.bfloat16 and x.dtype == dy.dtype and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and _wgrad_native_ok(dy, x)):
        return None
    return WgradRequest(x, w, stride, padding, w_param)


def _dual_call(Cn, wg: Optional[WgradRequest], dyc: torch.Tensor, w: torch.Tensor, ph: int, pw: int, bm: int,
               bn: int, splits: int, **kw) -> torch.Tensor:
    """conv_dgrad, or conv_dgrad_wgrad with ``wg``'s weight gradient in the same launch (sets wg.dw)."""
    if wg is None:
        return Cn.conv_dgrad(dyc, w, ph, pw, bm, bn, splits, **kw)
    defer = _can_defer(wg.w_param)
    pl = _plan("wgrad_dual", dyc.shape[0] * dyc.shape[2] * dyc.shape[3], dyc.shape[1], wg.x.shape[1], wg.R, wg.S,
               wg.stride[0])
    _native.count("wgrad")
    _native.count("wgrad_dual")
    dx, wg.dw = Cn.conv_dgrad_wgrad(dyc, w, ph, pw, bm, bn, splits, wg_x=wg.x, wg_R=wg.R, wg_S=wg.S,
                                    wg_sh=wg.stride[0], wg_sw=wg.stride[1], wg_ph=wg.padding[0], wg_pw=wg.padding[1],
                                    wg_splits=pl[2] if pl is not None else -1, wg_defer=defer,
                                    order=(pl[4] if pl is not None and pl[4] >= 0 and _DUAL == "2"
                                           else (1 if _DUAL == "2" else 0)), **kw)
    if defer:
        _defer_state["pending"] = True
    return dx


def _dgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride, padding,
           addend: Optional[torch.Tensor] = None, bn: Optional[BNGradLink] = None,
           wg: Optional[WgradRequest] = None) -> torch.Tensor:
    """dX (+ addend: the identity-shortcut gradient of a residual block, fused into the store).
    ``bn``: the producing BN layer's link — when the native kernel runs, it returns dz = dX·mask
    with the BN reduce done (``bn.dz`` is set).  ``wg``: this conv's weight gradient, computed in
    the same launch when the native kernel runs (``wg.dw`` is set)."""
    R, S = w.shape[2], w.shape[3]
    H, W = x.shape[2], x.shape[3]
    # stride 2 (ResNet's strided 3x3): the 4 output-phase sub-convolutions in one launch (needs an
    # even dX whose forward output is dY — true for every ResNet downsampling conv)
    s2 = (tuple(stride) == (2, 2) and R > 1 and H % 2 == 0 and W % 2 == 0 and dy.shape[2] * 2 == H
          and dy.shape[3] * 2 == W and (H + 2 * padding[0] - R) // 2 + 1 == dy.shape[2]
          and (W + 2 * padding[1] - S) // 2 + 1 == dy.shape[3])
    if ((tuple(stride) == (1, 1) or s2) and dy.shape[1] % 64 == 0 and w.shape[1] % 8 == 0 and padding[0] <= R - 1
            and padding[1] <= S - 1 and _native.use_native(dy, op="dgrad")):
        # stride 1: dX = conv(dY, flip(W) with C <-> K), padding R-1-p — conv_igemm.hip's DGRAD mode
        # reads the forward filter flipped and transposed in-kernel (no filter copy)
        dyc = dy.contiguous(memory_format=torch.channels_last)
        if addend is not None:
            addend = addend.to(dy.dtype).contiguous(memory_format=torch.channels_last)
        _native.count("dgrad_strided" if s2 else "dgrad")
        geo = dict(stride=2, H=H, W=W) if s2 else {}
        if bn is not None and not bn.used and bn.yc.dtype == dy.dtype:
            bn.used = True
            _native.count("dgrad_bn_fused")
            # (mode 2 or an addend: the full-register kernel variant, tuned under its own key)
            op = "dgrad_bnb2" if (bn.mode == 2 or addend is not None) else "dgrad_bnb"
            pl = _plan(op, x.shape[0] * H * W, w.shape[1], w.shape[0], R, S, stride[0]) or (-1, -1, -1, 0)
            bn.dz = _dual_call(_native.native(), wg, dyc, w, padding[0], padding[1], pl[0], pl[1], pl[2],
                               addend=addend, bn_x=bn.yc, bn_y=x if bn.mode == 2 else None, bn_w=bn.bn_w,
                               bn_b=bn.bn_b, bn_mean=bn.mean, bn_invstd=bn.invstd, bn_mode=bn.mode,
                               bn_sums=bn.sums, stages=pl[3], **geo)
            return bn.dz
        pl = _plan("dgrad", x.shape[0] * H * W, w.shape[1], w.shape[0], R, S, stride[0]) or (-1, -1, -1, 0)
        return _dual_call(_native.native(), wg, dyc, w, padding[0], padding[1], pl[0], pl[1], pl[2], addend=addend,
                          stages=pl[3], **geo)
    if (R == 1 and S == 1 and tuple(padding) == (0, 0) and dy.shape[1] % 64 == 0 and w.shape[1] % 8 == 0
            and _native.use_native(dy, op="dgrad")):
        # 1x1 stride-s (ResNet downsample): dY·W on the output grid is the stride-1 DGRAD GEMM; one
        # pass scatters it to every s-th input pixel, zeros elsewhere, + addend (the vendor path
        # ran a zero-fill kernel, its own dgrad, and autograd a separate add)
        Cn = _native.native()
        _native.count("dgrad_strided1x1")
        pl = _plan("dgrad", dy.shape[0] * dy.shape[2] * dy.shape[3], w.shape[1], w.shape[0], 1, 1, 1) or (-1, -1, -1, 0)
        comp = _dual_call(Cn, wg, dy.contiguous(memory_format=torch.channels_last), w, 0, 0, pl[0], pl[1], pl[2],
                          stages=pl[3])
        if addend is not None:
            addend = addend.to(dy.dtype).contiguous(memory_format=torch.channels_last)
        return Cn.upsample_add(comp, addend, x.shape[2], x.shape[3], stride[0], stride[1])
    _native.count("dgrad_vendor")
    dx = torch.ops.aten.convolution_backward(dy, x, w, None, list(stride), list(padding), [1, 1], False, [0, 0], 1,
                                             [True, False, False])[0]
    return dx if addend is None else dx + addend


FUSE_SHORTCUT_GRAD = os.environ.get("HYPERION_RESIDUAL_LINK", "1") == "1"  # models create ResidualLinks only when set (A/B)

# BN apply + ReLU fused into the consuming conv's operand read (conv_igemm.hip XF); A/B switch
# HYPERION_CONV_XF: "0" off, "1x1" only 1x1 consumers (each element transformed once), "all" every
# stride-1 consumer (a 3x3 re-transforms every element per tap)
_XF_MODE = os.environ.get("HYPERION_CONV_XF", "0")
FUSE_BN_APPLY = _XF_MODE in ("1", "all", "1x1")
XF_ONLY_1X1 = _XF_MODE == "1x1"
# launch plan of a fused consumer with >= 256 output channels (measured best, scripts/xf_bench.py);
# None: the plain conv's plan
XF_TILE = (128, 128, 1, 2)


class PendingBN:
    """A deferred ``relu(BN(y))``: the producer stored the raw conv output ``yc`` and its statistics
    sums; ``out`` (the activation autograd knows) and ``stats`` (save_mean / save_invstd) are
    allocated but written only by the consumer — the XF conv, or :func:`materialize` when the
    consumer cannot fuse.  Reached as ``out.grad_fn.bnpend``."""

    __slots__ = ("yc", "sums", "bn_w", "bn_b", "rm", "rv", "momentum", "eps", "stats", "out", "done")

    def __init__(self, yc, sums, bn_w, bn_b, rm, rv, momentum, eps, stats, out):
        self.yc, self.sums, self.bn_w, self.bn_b, self.rm, self.rv = yc, sums, bn_w, bn_b, rm, rv
        self.momentum, self.eps, self.stats, self.out = momentum, eps, stats, out
        self.done = False

    def release(self) -> None:
        # consumed: drop the tensors (``out`` would otherwise keep a ctx -> output -> grad_fn cycle)
        self.done = True
        self.yc = self.sums = self.bn_w = self.bn_b = self.rm = self.rv = self.stats = self.out = None


def pending_of(x: torch.Tensor) -> Optional[PendingBN]:
    p = getattr(x.grad_fn, "bnpend", None) if x.grad_fn is not None else None
    if p is None or p.done:
        return None
    if p.out.data_ptr() != x.data_ptr() or p.out.shape != x.shape:
        materialize(p)  # a view of the deferred output reached a consumer: apply the BN for real
        return None
    return p


def materialize(p: PendingBN) -> None:
    """Run a deferred BN apply as the standalone pass (the consumer is not an XF conv)."""
    if p.done:
        return
    _native.count("bn_apply_materialized")
    out, mean, invstd = _native.native().bn_fwd_sums(p.yc, None, p.sums, p.bn_w, p.bn_b, p.rm, p.rv, p.momentum,
                                                     p.eps, True)
    # (.data: filling the allocated-but-unwritten tensors is not a modification autograd must see —
    # the producer saved the stats views for its backward)
    p.out.data.copy_(out)
    p.stats.data[0].copy_(mean)
    p.stats.data[1].copy_(invstd)
    p.release()


def xf_consumer_ok(conv: nn.Conv2d) -> bool:
    """Can ``conv`` consume a deferred BN + ReLU (stride 1, "same" padding, <= 512 input channels)?"""
    R, S = conv.kernel_size
    return (FUSE_BN_APPLY and not isinstance(conv.padding, str) and tuple(conv.stride) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1 and conv.bias is None
            and tuple(conv.padding) == ((R - 1) // 2, (S - 1) // 2) and R % 2 == 1 and S % 2 == 1
            and conv.in_channels % 64 == 0 and conv.in_channels <= 512 and (R == 1 or not XF_ONLY_1X1))


def residual_link(x: torch.Tensor) -> Optional["ResidualLink"]:
    return ResidualLink(x) if FUSE_SHORTCUT_GRAD else None


class ResidualLink:
    """Carries a bottleneck's identity-shortcut gradient from its last conv/BN (which would return
    it as the residual input's gradient) to its first conv's data gradient, where the conv kernel
    adds it in the store epilogue — autograd's separate ``dx_conv1 + d_identity`` add kernel (one
    launch and two extra passes over the block input per block) disappears.

    Valid because both ops consume the SAME tensor (the block input) and the first op's backward
    always runs after the last op's (it depends on it through the main branch): the gradient only
    moves between two paths that autograd would have summed.  ``armed`` is set only when the
    first op took the fused path, so a fallback op never drops the gradient; and the last op
    parks its gradient only when the engine WILL run the first op's node in the same backward
    (``torch._C._will_engine_execute_node``) — a partial backward (``autograd.grad`` w.r.t. some
    leaves only, ``retain_graph=True``) gets the plain per-op gradients.
    """

    __slots__ = ("_src", "armed", "dres", "first_node")

    def __init__(self, src: torch.Tensor):
        # held weakly: the link rides ctx attributes (not saved tensors), so a strong reference
        # would keep one activation per layer alive under activation checkpointing
        self._src = weakref.ref(src)
        self.armed = False
        self.dres: Optional[torch.Tensor] = None
        self.first_node = None

    @property
    def src(self) -> Optional[torch.Tensor]:
        return self._src()


class BranchSumLink:
    """Sums the two data gradients of a downsampling block's input — its ``downsample`` conv and
    its first conv both read the block input, and autograd would add their gradients with a
    separate kernel (two full passes over the block input).  Whichever of the two backward calls
    runs first parks its dX here (tagged with its consumer index); the second one adds it in its
    own store (the conv kernel's addend epilogue, or the strided-dgrad scatter pass) and returns
    the sum, the first returns None.  Armed only when BOTH convs took the fused path in the
    forward (``users == 2``), so a fallback op never loses its gradient, and a node parks only
    when the engine will run the OTHER consumer's node in the same backward (a partial
    ``autograd.grad`` that reaches one consumer returns plain per-op gradients; a parked tensor
    from an earlier, abandoned pass is dropped by its own owner).  Reference: torchvision
    ``Bottleneck.forward`` (``out += identity``).
    """

    __slots__ = ("_src", "users", "pending", "nodes")

    def __init__(self, src: torch.Tensor):
        self._src = weakref.ref(src)  # weakly, as ResidualLink
        self.users = 0
        self.pending = None  # (owner consumer index, dX)
        self.nodes = [None, None]  # grad_fn of each consumer's output

    @property
    def src(self) -> Optional[torch.Tensor]:
        return self._src()


def branch_sum_link(x: torch.Tensor) -> Optional[BranchSumLink]:
    return BranchSumLink(x) if FUSE_SHORTCUT_GRAD else None


# Deferred weight-gradient reduce: a split-K weight gradient's reduce kernel is not launched; it rides
# on the NEXT conv_wgrad launch as extra workgroups (csrc/kernels/conv_wgrad.hip WgradPendingReduce),
# ~50 launches fewer per ResNet-50 backward.  Safe only when nothing reads the gradient before that
# launch: the weight must be a leaf whose .grad is None (AccumulateGrad steals the tensor — no add
# or cast kernel reads it), and every in-backward reader of .grad (DDP / FSDP gradient hooks) calls
# flush_wgrad() first; the last pending reduce runs at the end of the backward pass (engine callback).
DEFER_WGRAD_REDUCE = os.environ.get("HYPERION_WGRAD_DEFER", "1") == "1"
_defer_state = {"pending": False, "queued": False}

# Where a layer's weight gradient runs (HYPERION_WGRAD_FUSE):
# * "dgrad" (default): in the layer's own data-gradient launch (csrc/kernels/conv_dual.hip);
# * "bn": PARKED until the next BatchNorm dx pass of the backward (the layer below) and run in that
#   pass's launch (csrc/kernels/bn_wgrad.hip), the data gradients keeping their own kernels —
#   measured no faster than separate launches (4.80 vs 4.79 ms; "dgrad" 4.67, profiles/r05/
#   dual_ab.txt): every workgroup of the fused launch takes the larger register / LDS footprint,
#   so the bandwidth-bound dx blocks lose the occupancy they stream with;
# * "0": its own launch.
# A parked gradient is handed to autograd unwritten, so the same rules as the deferred reduce apply
# (``_can_defer``: a leaf whose .grad is None — stolen, never read before the flush), and every
# in-backward reader flushes first (flush_wgrad: DDP / FSDP hooks, the end-of-backward callback).
WGRAD_FUSE = os.environ.get("HYPERION_WGRAD_FUSE", "dgrad")


class _ParkedWgrad:
    """A parked weight gradient.  Its output is held by STORAGE, not as a tensor: a second tensor
    reference would stop AccumulateGrad from stealing the gradient — it would clone the
    not-yet-written values instead (the deferred reduce's rule, conv_ops.cpp PendingWgrad)."""

    __slots__ = ("dy", "x", "R", "S", "stride", "padding", "store", "meta", "plan")

    def __init__(self, dy, x, w, stride, padding, dw, plan):
        self.dy, self.x, self.R, self.S = dy, x, w.shape[2], w.shape[3]
        self.stride, self.padding, self.plan = tuple(stride), tuple(padding), plan
        self.store = dw.untyped_storage()
        self.meta = (dw.dtype, dw.device, dw.storage_offset(), tuple(dw.shape), tuple(dw.stride()))

    @property
    def dw(self) -> torch.Tensor:
        """A fresh tensor over the parked output's storage (the kernel writes through it)."""
        dt, dev, off, shape, stride = self.meta
        return torch.empty(0, dtype=dt, device=dev).set_(self.store, off, shape, stride)


_parked: dict = {"req": None}


def _fused_wgrad_tile(plan) -> tuple:
    """(bm, bn, splits) of a parked weight gradient from its tuned standalone plan: the fused launch
    runs 64 x 64 / 128 x 64 / 64 x 128 tiles (a 128 x 128 plan becomes 128 x 64, same splits)."""
    if plan is None:
        return 64, 64, -1
    bm, bn, splits = plan[0], plan[1], plan[2]
    if bm not in (64, 128) or bn not in (64, 128):
        return 64, 64, -1
    if bm == 128 and bn == 128:
        bn = 64
    return bm, bn, splits


def _flush_parked() -> None:
    """Run a parked weight gradient in its own launch (nobody consumed it); its split-K reduce is
    deferred into the next weight-gradient launch or the final flush."""
    req, _parked["req"] = _parked["req"], None
    if req is None:
        return
    bm, bn, splits = _fused_wgrad_tile(req.plan)
    _native.native().conv_wgrad(req.dy, req.x, req.R, req.S, req.stride[0], req.stride[1], req.padding[0],
                                req.padding[1], bm, bn, splits, defer=True, out=req.dw)
    _defer_state["pending"] = True


def _park_ok(dy: torch.Tensor, x: torch.Tensor, w_param: Optional[torch.Tensor]) -> bool:
    return (WGRAD_FUSE == "bn" and not _streams.enabled() and dy.dtype == torch.bfloat16 and x.dtype == dy.dtype
            and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and dy.is_contiguous(memory_format=torch.channels_last) and _wgrad_native_ok(dy, x)
            and _can_defer(w_param))


def _park_wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride, padding) -> torch.Tensor:
    """Park this layer's weight gradient (caller checked :func:`_park_ok`); returns its dW tensor,
    written by the launch that consumes the request (or a flush)."""
    _flush_parked()  # one slot: an earlier request nobody consumed runs now
    _native.count("wgrad")
    dw = torch.empty(w.shape, dtype=x.dtype, device=x.device).contiguous(memory_format=torch.channels_last)
    P, Q = dy.shape[2], dy.shape[3]
    plan = _plan("wgrad", dy.shape[0] * P * Q, dy.shape[1], x.shape[1], w.shape[2], w.shape[3], stride[0])
    _parked["req"] = _ParkedWgrad(dy, x, w, stride, padding, dw, plan)
    _defer_state["pending"] = True
    return dw


def _bn_dx(C, dout, yc, bn_w, mean, invstd, sums):
    """The BN dx pass (dz already masked, sums complete), carrying the parked weight gradient of the
    layer above when there is one."""
    req = _parked["req"]
    if req is None or dout.dtype != torch.bfloat16:
        return C.bn_bwd_dx(dout, yc, bn_w, mean, invstd, True, sums)
    _parked["req"] = None
    bm, bn, splits = _fused_wgrad_tile(req.plan)
    _native.count("wgrad_bn_fused")
    dyc, dbw, dbb, _ = C.bn_bwd_dx_wgrad(dout, yc, bn_w, mean, invstd, True, sums, wg_dy=req.dy, wg_x=req.x,
                                         wg_R=req.R, wg_S=req.S, wg_sh=req.stride[0], wg_sw=req.stride[1],
                                         wg_ph=req.padding[0], wg_pw=req.padding[1], wg_bm=bm, wg_bn=bn,
                                         wg_splits=splits, wg_defer=True, wg_out=req.dw)
    _defer_state["pending"] = True
    return dyc, dbw, dbb


def flush_wgrad() -> None:
    """Run a parked weight gradient and a deferred weight-gradient reduce now (no-op when none)."""
    _defer_state["queued"] = False
    if _parked["req"] is not None:
        _flush_parked()
    if _defer_state["pending"]:
        _defer_state["pending"] = False
        _native.native().conv_wgrad_flush()


def _can_defer(w_param: Optional[torch.Tensor]) -> bool:
    # (grad mode off: a create_graph backward would make AccumulateGrad clone, not steal)
    if not (DEFER_WGRAD_REDUCE and w_param is not None and w_param.grad is None and not _streams.enabled()
            and not torch.is_grad_enabled()):
        return False
    # a tensor hook on the weight sees dw before AccumulateGrad (and before any flush): its values
    # must be final, so no deferral.  (Post-accumulate hooks — DDP / FSDP — call flush_wgrad first.)
    if getattr(w_param, "_backward_hooks", None):
        return False
    if not _defer_state["queued"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush_wgrad)
        except RuntimeError:  # not inside a backward pass: nobody would flush
            return False
        _defer_state["queued"] = True
    return True


def _wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride, padding,
           w_param: Optional[torch.Tensor] = None) -> torch.Tensor:
    # csrc/kernels/conv_wgrad.hip: split-K MFMA GEMM over the output pixels with transposed LDS
    # reads (one kernel + one deterministic partial-sum/cast kernel; MIOpen used 3-4 launches).
    # (hipBLASLt on the 1x1 case dYᵀ·X runs a 10⁵-long reduction without split-K: 10x slower.)
    R, S = w.shape[2], w.shape[3]
    P, Q = dy.shape[2], dy.shape[3]
    if _wgrad_native_ok(dy, x):
        dyc = dy.contiguous(memory_format=torch.channels_last)
        _native.count("wgrad")
        defer = _can_defer(w_param)
        pl = _plan("wgrad", dy.shape[0] * P * Q, dy.shape[1], x.shape[1], R, S, stride[0]) or (-1, -1, -1, 0)
        dw = _native.native().conv_wgrad(dyc, x, R, S, stride[0], stride[1], padding[0], padding[1], pl[0], pl[1],
                                         pl[2], defer=defer)
        if defer:
            _defer_state["pending"] = True
        return dw
    _native.count("wgrad_vendor")
    return torch.ops.aten.convolution_backward(dy, x, w, None, list(stride), list(padding), [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


def _will_run(ref) -> bool:
    """``ref``: a weakref to a consumer's backward node (weak: the node's ctx holds the link)."""
    node = ref() if ref is not None else None
    return node is not None and torch._C._will_engine_execute_node(node)


class _ConvBNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bn_w, bn_b, rm, rv, residual, stride, padding, momentum, eps, act, link_in, link_out,
                branch, bidx, prod, xin=None, defer=False):
        C = _native.native()
        # BN statistics: the conv epilogue ADDS Σy, Σy² into a zeroed [2, K] slice of the forward's
        # arena; the apply finalizes inline.  The backward's Σdz, Σdz·x slice is reserved now so
        # it shares the same single zero-fill.
        K = w.shape[0]
        sums = _native.zeroed(_native.STAT_SLOTS * 2 * K, x.device)
        ctx.bsums = _native.zeroed(_native.STAT_SLOTS * 2 * K, x.device)
        P = (x.shape[2] + 2 * padding[0] - w.shape[2]) // stride[0] + 1
        Q = (x.shape[3] + 2 * padding[1] - w.shape[3]) // stride[1] + 1
        pl = _plan("fwd", x.shape[0] * P * Q, K, x.shape[1], w.shape[2], w.shape[3], stride[0]) or (-1, -1, -1, 0)
        if xin is not None:
            # x is the deferred activation of the producing layer: read its raw conv output, apply
            # that layer's BN + ReLU on the operand path, and fill x (and its BN stats) on the way.
            # Tile: 128x128 / 2 stages where the output has >= 256 channels (measured best for the
            # fused 1x1 consumers, scripts/xf_bench.py), else the plain conv's plan
            if XF_TILE is not None and K >= 256 and K % 128 == 0:
                pl = XF_TILE
            _native.count("conv_xf")
            yc, _, _ = C.conv_fwd(xin.yc, w, stride[0], stride[1], padding[0], padding[1], True, pl[0], pl[1], pl[2],
                                  sums=sums, stages=pl[3], xf_sums=xin.sums, xf_w=xin.bn_w, xf_b=xin.bn_b,
                                  xf_rm=xin.rm, xf_rv=xin.rv, xf_momentum=xin.momentum, xf_eps=xin.eps, xf_out=x,
                                  xf_stats=xin.stats)
            xin.release()
        else:
            yc, _, _ = C.conv_fwd(x, w, stride[0], stride[1], padding[0], padding[1], True, pl[0], pl[1], pl[2],
                                  sums=sums, stages=pl[3])
        if residual is not None:
            residual = residual.to(x.dtype).contiguous(memory_format=torch.channels_last)
        if defer:
            # no apply pass: the consumer conv applies BN + ReLU as it reads yc (PendingBN)
            out = torch.empty_like(yc)
            stats = torch.empty(2, K, device=yc.device, dtype=torch.float32)
            mean, invstd = stats[0], stats[1]
            ctx.bnpend = PendingBN(yc, sums, bn_w, bn_b, rm, rv, momentum, eps, stats, out)
        else:
            out, mean, invstd = C.bn_fwd_sums(yc, residual, sums, bn_w, bn_b, rm, rv, momentum, eps, act)
        # without a residual the backward recomputes the ReLU mask from yc (no need to keep `out`)
        ctx.save_for_backward(x, w, yc, out if (act and residual is not None) else None, bn_w, bn_b, mean, invstd)
        ctx.cfg = (stride, padding, act, residual is not None)
        ctx.links = (link_in, link_out, branch, bidx)
        ctx.prod = prod  # the BNGradLink of the fused layer that produced x (or None)
        ctx.w_param = w if (w.is_leaf and w.requires_grad) else None  # (deferred wgrad reduce)
        # this layer's own link for the conv that will consume `out` (reached as out.grad_fn.bnlink)
        mode = (2 if residual is not None else 1) if act else 0
        ctx.bnlink = (BNGradLink(yc, bn_w, bn_b, mean, invstd, mode, ctx.bsums)
                      if FUSE_BN_BACKWARD and mode in FUSE_BN_MODES else None)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, yc, out, bn_w, bn_b, mean, invstd = ctx.saved_tensors
        stride, padding, act, has_res = ctx.cfg
        link_in, link_out, branch, bidx = ctx.links
        need_res = has_res and ctx.needs_input_grad[6]
        bsums, ctx.bsums = ctx.bsums, None  # a second backward (retain_graph) takes fresh zeros
        own = ctx.bnlink
        if own is not None and own.dz is not None and dout is own.dz:
            # the consumer's dgrad epilogue already masked dout and summed Σdz, Σdz·x: dx pass only
            # (carrying the parked weight gradient of the layer above, WGRAD_FUSE "bn")
            dyc, dbw, dbb = _bn_dx(_native.native(), dout, yc, bn_w, mean, invstd, own.sums)
            dres = dout if need_res else None
        else:
            if own is not None and own.used:
                bsums = None  # the epilogue ran into these sums, but its dz is not all of dout
            dyc, dres, dbw, dbb = _native.native().bn_bwd(dout, yc, out, bn_w, bn_b, mean, invstd, True, act,
                                                          need_res, sums=bsums)
        if own is not None:
            own.dz, own.used = None, True  # consumed: a retained-graph second backward takes the full path
        if need_res and link_out is not None and link_out.armed and _will_run(link_out.first_node):
            link_out.dres, dres = dres, None  # added by the block's first conv dgrad instead
        add = None
        if link_in is not None and link_in.dres is not None:
            add, link_in.dres = link_in.dres, None
        dw = None
        if ctx.needs_input_grad[1] and _streams.use_side_for(w):
            # off the critical path: forked BEFORE the data gradient, so the two overlap
            dw = _streams.run_on_side(lambda: _wgrad(dyc, x, w, stride, padding), [dyc, x], dyc.device)
        dx = None
        prod = ctx.prod
        # this layer's weight gradient: parked for the next BN dx pass (WGRAD_FUSE "bn"), or in the
        # data gradient's launch ("dgrad"), or its own launch
        park = dw is None and ctx.needs_input_grad[1] and _park_ok(dyc, x, ctx.w_param)
        wg = (wgrad_request(dyc, x, w, stride, padding, ctx.w_param)
              if dw is None and not park and ctx.needs_input_grad[1] and ctx.needs_input_grad[0] else None)
        if ctx.needs_input_grad[0]:
            if branch is not None and branch.users == 2 and _will_run(branch.nodes[1 - bidx]):
                pend, branch.pending = branch.pending, None
                if pend is not None and pend[0] == bidx:
                    pend = None  # our own dX from an abandoned pass (its partner never ran): stale
                if pend is None:  # first of the block input's two consumers: park dX for the second
                    branch.pending = (bidx, _dgrad(dyc, x, w, stride, padding, addend=add, wg=wg))
                else:  # the second computes the whole gradient of x: it can run the BN epilogue
                    other = pend[1]
                    dx = _dgrad(dyc, x, w, stride, padding, addend=other if add is None else other + add, bn=prod,
                                wg=wg)
            else:
                # the whole gradient of x unless another op consumes x outside our links (then the
                # producer sees a summed gradient and takes its full path)
                dx = _dgrad(dyc, x, w, stride, padding, addend=add, bn=prod, wg=wg)
        if dw is None and park:
            dw = _park_wgrad(dyc, x, w, stride, padding)
        if dw is None and wg is not None and wg.dw is not None:
            dw = wg.dw
        if dw is None and ctx.needs_input_grad[1]:
            dw = _wgrad(dyc, x, w, stride, padding, w_param=ctx.w_param)
        return (dx, dw, dbw if ctx.needs_input_grad[2] else None, dbb if ctx.needs_input_grad[3] else None, None, None,
                dres, None, None, None, None, None, None, None, None, None, None, None, None)


def _xf_fusable(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor, residual, link, branch) -> bool:
    """Will conv_bn_act take the native fused path for (conv, bn, x) with an XF-capable geometry
    (so a pending BN on x is applied by this conv's operand read)?"""
    wdt = conv.weight.dtype
    if x.is_cuda and torch.is_autocast_enabled(x.device.type):
        wdt = torch.get_autocast_dtype(x.device.type)  # conv_bn_act casts the weight (and x) to it
        if wdt != x.dtype:
            return False
    if not (xf_consumer_ok(conv) and bn.training and bn.track_running_stats and bn.momentum is not None
            and bn.affine and x.is_cuda and x.dtype == torch.bfloat16 and wdt == x.dtype
            and _native.use_native(x, op="conv") and _native.use_native(x, op="bn")):
        return False
    if (link is not None and x is link.src) or (branch is not None and x is branch.src):
        return False  # a block input is never a deferred activation
    return _native_conv_ok(x, conv, conv.weight, wdt=wdt) and not _is_stem(conv, x)


def _eval_affine(bn: nn.Module, device):
    """Eval-mode BN as a per-channel affine (scale = γ/sqrt(running_var + eps), shift = β -
    running_mean·scale, fp32), cached on the module until its statistics or parameters change."""
    ts = (bn.running_mean, bn.running_var, bn.weight, bn.bias)
    key = tuple((t.data_ptr(), t._version) if t is not None else None for t in ts)
    cache = bn.__dict__.get("_hyp_eval_affine")
    if cache is not None and cache[0] == key:
        return cache[1], cache[2]
    with torch.no_grad():
        inv = torch.rsqrt(bn.running_var.float() + bn.eps)
        sc = inv * bn.weight.float() if bn.weight is not None else inv
        sh = -bn.running_mean.float() * sc
        if bn.bias is not None:
            sh = sh + bn.bias.float()
        sc, sh = sc.contiguous(), sh.contiguous()
    bn.__dict__["_hyp_eval_affine"] = (key, sc, sh)
    return sc, sh


def _inference_weight(conv: nn.Conv2d, dt: torch.dtype) -> torch.Tensor:
    """The conv weight in ``dt`` for a no-grad forward, cast once and cached (autocast would re-cast
    the fp32 weight on every call)."""
    w = conv.weight
    if w.dtype == dt:
        return w
    key = (dt, w.data_ptr(), w._version)
    cache = conv.__dict__.get("_hyp_cast")
    if cache is None or cache[0] != key:
        with torch.no_grad():
            cache = (key, w.to(dt).contiguous(memory_format=torch.channels_last))
        conv.__dict__["_hyp_cast"] = cache
    return cache[1]


def _conv_bn_eval(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor,
                  residual: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Inference: conv → BN(running stats) → (+ residual) → (ReLU) as ONE launch — the BN folded into
    the conv kernel's epilogue as a per-channel affine (``conv_fwd_affine``; the split-K reduce
    carries the same epilogue).  None when outside the kernel's envelope."""
    if bn.training or not bn.track_running_stats or bn.running_mean is None:
        return None
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (x, conv.weight, bn.weight,
                                                                                      bn.bias, residual)):
        return None  # eval-mode training (frozen BN): the autograd path below
    if not (x.is_cuda and _native.use_native(x, op="conv") and _native.use_native(x, op="bn")):
        return None
    dt = x.dtype
    if torch.is_autocast_enabled(x.device.type):
        dt = torch.get_autocast_dtype(x.device.type)
    if dt == torch.float32:  # fp32: the BN folded into the fp32-MFMA GEMM (ops/conv_f32.py), when faster
        from .conv_f32 import conv_bn_eval_f32

        sc, sh = _eval_affine(bn, x.device)
        return conv_bn_eval_f32(conv, bn, x, residual, sc, sh)
    if dt not in (torch.bfloat16, torch.float16):
        return None
    xc = x.to(dt) if x.dtype != dt else x
    w = _inference_weight(conv, dt)
    if not _native_conv_ok(xc, conv, w):
        return None
    if residual is not None:
        residual = residual.to(dt).contiguous(memory_format=torch.channels_last)
    sc, sh = _eval_affine(bn, x.device)
    _native.count("conv_bn_eval")
    return _native.native().conv_fwd_affine(xc, w, conv.stride[0], conv.stride[1], conv.padding[0], conv.padding[1],
                                            sc, sh, residual, bool(bn.act))


# ---- the RGB stem (7x7, stride 2, padding 3, C <= 4): csrc/kernels/stem.hip rewrites it as
# space-to-depth Xs [N, 16, P+3, Q+3] and a stride-1 R=4 conv whose 64-element reduction runs are 4
# adjacent Xs pixels (conv_fwd / conv_wgrad with a 16-element pixel stride); W4[k, dr, ds*16 +
# (2a+b)*C + c] = W[k, c, 2dr+a, 2ds+b] (zero for tap 7).
_STEM_IDX: dict = {}


def _stem_index(C: int, device) -> tuple:
    """(idx4 [256]: column of [W.view(K, C*49) | 0] feeding each W4 column, inv [C*49]: the W4
    column of each W element)."""
    key = (C, str(device))
    if key not in _STEM_IDX:
        idx4 = torch.full((4, 4, 16), C * 49, dtype=torch.long)  # the appended zero column
        inv = torch.empty(C * 49, dtype=torch.long)
        for dr in range(4):
            for ds in range(4):
                for a in range(2):
                    for b in range(2):
                        r, q = 2 * dr + a, 2 * ds + b
                        if r > 6 or q > 6:
                            continue
                        for c in range(C):
                            src = c * 49 + r * 7 + q
                            idx4[dr, ds, (2 * a + b) * C + c] = src
                            inv[src] = (dr * 4 + ds) * 16 + (2 * a + b) * C + c
        _STEM_IDX[key] = (idx4.reshape(-1).to(device), inv.to(device))
    return _STEM_IDX[key]


def stem_weight(w: torch.Tensor) -> torch.Tensor:
    """W [K, C, 7, 7] -> W4 [K, 64, 4, 1] (channels-last; memory [k][dr][ds*16 + (2a+b)*C + c]).
    Differentiable (an index gather): the rewritten conv's weight gradient flows back to W."""
    K, C = w.shape[0], w.shape[1]
    idx4, _ = _stem_index(C, w.device)
    wx = torch.nn.functional.pad(w.reshape(K, C * 49), (0, 1))
    w4 = wx.index_select(1, idx4).reshape(K, 4, 1, 64)
    return w4.permute(0, 3, 1, 2)


def stem_weight_grad(dw4: torch.Tensor, C: int) -> torch.Tensor:
    """dW [K, C, 7, 7] from dW4 [K, 64, 4, 1] (channels-last): each W element feeds one W4 column."""
    K = dw4.shape[0]
    _, inv = _stem_index(C, dw4.device)
    flat = dw4.permute(0, 2, 3, 1).reshape(K, 256)  # memory order [k][dr][64]
    return flat.index_select(1, inv).reshape(K, C, 7, 7)


def stem_s2d_reference(x: torch.Tensor) -> torch.Tensor:
    """PyTorch form of ``stem_s2d`` (the kernel's numerics oracle): x [N, C, H, W] -> Xs
    [N, 16, P+3, Q+3], Xs[n, (2a+b)*C + c, i, j] = x_pad3[n, c, 2i+a, 2j+b]."""
    N, C, H, W = x.shape
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    Hs, Ws = P + 3, Q + 3
    xp = torch.nn.functional.pad(x, (3, 2 * Ws - W - 3, 3, 2 * Hs - H - 3))
    xs = xp.reshape(N, C, Hs, 2, Ws, 2).permute(0, 2, 4, 3, 5, 1).reshape(N, Hs, Ws, 4 * C)
    xs = torch.nn.functional.pad(xs, (0, 16 - 4 * C))
    return xs.permute(0, 3, 1, 2)


def stem_runs_reference(xs: torch.Tensor) -> torch.Tensor:
    """What the kernels read with a 16-element pixel stride: X4 [N, 64, P+3, Q], X4[n, ds*16 + e, i, q]
    = Xs[n, e, i, q + ds] — so the stem is F.conv2d(X4, W4) (used by the CPU check of the rewrite)."""
    Q = xs.shape[3] - 3
    return torch.cat([xs[:, :, :, ds:ds + Q] for ds in range(4)], dim=1)


def _is_stem(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (3, 3)
            and conv.groups == 1 and tuple(conv.dilation) == (1, 1) and conv.bias is None
            and x.dim() == 4 and 1 <= x.shape[1] <= 4 and not x.requires_grad
            and x.dtype in (torch.bfloat16, torch.float16) and x.is_cuda and conv.out_channels % 8 == 0)


class _StemConvBNActFn(torch.autograd.Function):
    """stem conv -> BN (training) -> ReLU on the native kernels; no input gradient (the image)."""

    @staticmethod
    def forward(ctx, x, w, bn_w, bn_b, rm, rv, momentum, eps, act):
        C = _native.native()
        K, Cin = w.shape[0], w.shape[1]
        xs = C.stem_s2d(x.contiguous(memory_format=torch.channels_last))
        w4 = C.stem_weight4(w.detach())  # == stem_weight(w) in one launch
        sums = _native.zeroed(_native.STAT_SLOTS * 2 * K, x.device)
        ctx.bsums = _native.zeroed(_native.STAT_SLOTS * 2 * K, x.device)
        yc = C.stem_conv_fwd(xs, w4, sums)
        out, mean, invstd = C.bn_fwd_sums(yc, None, sums, bn_w, bn_b, rm, rv, momentum, eps, act)
        ctx.save_for_backward(xs, yc, bn_w, bn_b, mean, invstd)
        ctx.cfg = (Cin, act)
        # the gradient in the weight's own layout (AccumulateGrad then steals it: no copy kernel)
        ctx.w_cl = not w.is_contiguous() and w.is_contiguous(memory_format=torch.channels_last)
        return out

    @staticmethod
    def backward(ctx, dout):
        xs, yc, bn_w, bn_b, mean, invstd = ctx.saved_tensors
        Cin, act = ctx.cfg
        bsums, ctx.bsums = ctx.bsums, None
        C = _native.native()
        dyc, _, dbw, dbb = C.bn_bwd(dout.contiguous(memory_format=torch.channels_last), yc, None, bn_w, bn_b, mean,
                                    invstd, True, act, False, sums=bsums)
        dw = None
        if ctx.needs_input_grad[1]:
            _native.count("wgrad")
            dw4 = C.stem_conv_wgrad(dyc, xs).contiguous(memory_format=torch.channels_last)
            dw = C.stem_weight4_grad(dw4, Cin, ctx.w_cl)  # == stem_weight_grad(dw4, Cin), one launch
        return (None, dw, dbw if ctx.needs_input_grad[2] else None, dbb if ctx.needs_input_grad[3] else None,
                None, None, None, None, None)


def conv_bn_act(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                link: Optional[ResidualLink] = None, branch: Optional[BranchSumLink] = None,
                defer: bool = False) -> torch.Tensor:
    """``bn(conv(x), residual)`` for a ``BatchNormAct2d`` ``bn``; fused on gfx950 when possible.

    ``link``: a ``ResidualLink`` whose ``src`` is the block input — pass it to the block's FIRST
    conv (``x is link.src``) and to its LAST (``residual is link.src``) to fuse the shortcut
    gradient into the first conv's data gradient.  ``branch``: a ``BranchSumLink`` on the block
    input, passed to the downsample conv and the first conv (sums their data gradients in-kernel).
    ``defer``: the output feeds a conv for which :func:`xf_consumer_ok` holds, called next through
    this function — BN + ReLU are then applied by that conv's operand read (no apply pass); any
    other consumer must see the output materialized (this function does it for its own input)."""
    pend = pending_of(x)
    if pend is not None and not _xf_fusable(conv, bn, x, residual, link, branch):
        materialize(pend)
        pend = None
    if not bn.training:
        out = _conv_bn_eval(conv, bn, x, residual)
        if out is not None:
            return out
    w = conv.weight
    if x.is_cuda and torch.is_autocast_enabled(x.device.type):
        # autocast (the reference's fp16 / bf16 AMP trainers): run the fused kernels on the autocast
        # dtype like torch's conv would — x and the fp32 master weight cast once per call (the cast
        # is differentiable: dW flows back to the fp32 weight), BN parameters stay fp32
        dt = torch.get_autocast_dtype(x.device.type)
        if dt in (torch.bfloat16, torch.float16):
            if x.dtype != dt:
                x = x.to(dt)
                if residual is None and link is not None:
                    link = None  # the link tracks the caller's tensor, not this cast copy
                if branch is not None:
                    branch = None
            if w.dtype != dt:
                w = w.to(dt)
            if residual is not None and residual.dtype != dt:
                residual = residual.to(dt)
    stride, padding = tuple(conv.stride), tuple(conv.padding)
    use = (
        bn.training
        and bn.track_running_stats
        and bn.momentum is not None
        and bn.affine
        and _native.use_native(x, op="conv")
        and _native.use_native(x, op="bn")
    )
    if use and residual is None and link is None and branch is None and _is_stem(conv, x) and w.dtype == x.dtype:
        # the RGB stem: space-to-depth (stem.hip) + the 64-wide kernels with a 16-element pixel stride
        _native.count("stem_s2d")
        _native.count("conv_bn_act")
        bn._host_batches += 1
        return _native.apply_fn(_StemConvBNActFn, x, w, bn.weight, bn.bias, bn.running_mean, bn.running_var, float(bn.momentum),
                                      float(bn.eps), bool(bn.act))
    use = use and _native_conv_ok(x, conv, w)
    if not use:
        _native.count("conv_bn_act_fallback")
        return bn(conv(x), residual=residual)  # fp32: Conv2d routes to the native fp32 path (conv_f32)
    _native.count("conv_bn_act")
    bn._host_batches += 1  # BatchNormAct2d's host-side num_batches_tracked mirror
    link_in = link_out = None
    if link is not None:
        if x is link.src and residual is None:
            link.armed = True  # the first conv runs fused: its dgrad can take the shortcut gradient
            link_in = link
        elif residual is link.src and link.armed:
            link_out = link
    bidx = -1
    if branch is not None:
        if x is branch.src and branch.users < 2:
            bidx = branch.users
            branch.users += 1
        else:
            branch = None
    # x produced by another fused layer: its BN backward reduce can ride on our dgrad epilogue
    prod = getattr(x.grad_fn, "bnlink", None) if (FUSE_BN_BACKWARD and x.grad_fn is not None) else None
    defer = (defer and FUSE_BN_APPLY and bool(bn.act) and residual is None and torch.is_grad_enabled()
             and x.dtype == torch.bfloat16 and w.dtype == x.dtype and bn.num_features <= 512)
    out = _native.apply_fn(_ConvBNActFn, x, w, bn.weight, bn.bias, bn.running_mean, bn.running_var, residual,
                             stride, padding, float(bn.momentum), float(bn.eps), bool(bn.act),
                             link_in, link_out, branch, bidx, prod, pend, defer)
    if out.grad_fn is not None:  # (no graph under no_grad: nothing to link)
        if branch is not None:
            branch.nodes[bidx] = weakref.ref(out.grad_fn)
        if link_in is not None:
            link_in.first_node = weakref.ref(out.grad_fn)
    return out
