"""Data-parallel training with bucketed gradient all-reduce overlapped with backward.

Reference: ``torch.nn.parallel.DistributedDataParallel`` wrapped around every trainer model
(``distributed_utils.py:159,229,475``; SURVEY §2.2 "DP: DDP", K2-K6).

MI355X design:
* gradients are packed into persistent flat buckets the moment each parameter's gradient is
  final (``post_accumulate_grad`` hook), and a bucket's all-reduce (RCCL ``avg``) is issued as
  soon as it is complete — in bucket order on every rank — so RCCL traffic over xGMI overlaps the
  rest of the backward pass;
* buckets are **fp32 by default** whatever the compute dtype: the reference reduced fp32
  gradients, and a bf16 sum over 8 ranks keeps 8 significant bits.  A bf16/fp16
  parameter's gradient is up-converted by the pack copy and handed to the optimizer as
  ``param.main_grad`` (an fp32 bucket view; ``param.grad`` is released after packing, so the
  next backward's AccumulateGrad steals its fresh gradient instead of adding into it).
  ``comm_dtype=torch.bfloat16`` (opt-in) halves the bytes on the wire; ``comm_dtype=None`` uses
  each parameter's own dtype;
* bucket sizes default to 64 MiB (first bucket 4 MiB): with 288 GB HBM per GPU memory is no
  constraint, and on a fully-connected 8-GPU xGMI mesh RCCL's ring/direct algorithms reach
  their bus bandwidth only at tens of MiB per call, while a small first bucket
  lets the first all-reduce start early in backward;
* after backward, ``param.grad`` (same dtype) or ``param.main_grad`` (fp32 bucket, low-precision
  parameter) points at the bucket slice, so the fused optimizer reads the reduced gradient in
  place (no copy back) and its pointer table stays valid across steps;
* ``broadcast_buffers`` reproduces the reference's per-forward BN buffer broadcast (K5); under a
  segmented hipGraph capture it is an eager hole before the forward, so graphed steps keep it;
* a segmented capture of the whole step (``train/segments.py``, used by the trainers' captured
  step) records each bucket's all-reduce and its wait as eager holes at the points where the
  eager backward issued them: replays overlap RCCL with the rest of the backward for every model;
* ``defer_allreduce`` (set by ``TrainStep`` for hipGraph replay): backward only packs the buckets
  and ``allreduce_buckets()`` reduces them afterwards — the captured fwd+bwd graph and the
  optimizer graph then hold no RCCL call, and the collectives run eagerly between the two
  replays (one launch per bucket; no communication inside a captured graph);
* ``partial_backward`` / ``complete_buckets`` / ``allreduce_buckets(indices, wait=False)`` let a
  captured step split its backward in two graphs and reduce the buckets completed by the first
  (the top layers: most of the bytes) on the comm stream while the second replays.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import streams as _streams
from ..train import segments as _segments
from ..ops.conv import flush_wgrad as _flush_wgrad
from ..utils.nvtx import range_push, range_pop
from .comm import get_comm


def _flat_broadcast(tensors: List[torch.Tensor], src: int, group) -> None:
    """Broadcast a list of tensors as one flat message per dtype."""
    by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for ts in by_dtype.values():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off : off + n].view_as(t))
                off += n


def _param_view(flat: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """``flat`` (p.numel() elements) viewed with p's own strides when p is densely packed in some
    dimension order (channels-last conv weights): the gradient then has the parameter's layout
    (the fused optimizer needs grad and param element orders to match), else a plain view."""
    if p.is_contiguous():
        return flat.view(p.shape)
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last):
        return flat.as_strided(p.shape, p.stride())
    return flat.view(p.shape)


def _mt_ok(g: torch.Tensor, slot: torch.Tensor) -> bool:
    """The multi-tensor pack applies: same element order, 16-byte aligned, a native dtype."""
    from ..ops import _native

    return (g.is_cuda and g.shape == slot.shape and g.data_ptr() % 16 == 0 and g.dtype in _native.DTYPE_CODE
            and slot.dtype in _native.DTYPE_CODE and _native.use_native(g, op="copy_mt")
            and all(sa == sb for sa, sb, n in zip(g.stride(), slot.stride(), g.shape) if n > 1)
            and (g.is_contiguous() or g.is_contiguous(memory_format=torch.channels_last)))


class _Bucket:
    __slots__ = ("index", "params", "offsets", "buf", "ready", "got", "work", "launched")

    def __init__(self, index: int, params: List[nn.Parameter], dtype: torch.dtype, device: torch.device):
        self.index = index
        self.params = params
        self.offsets: List[int] = []
        # every slot starts on a 64-byte boundary: the fused optimizer's vector loads (and its
        # table builder) need >= 16-byte aligned gradients; the padding stays zero
        align = max(1, 64 // torch.empty((), dtype=dtype).element_size())
        off = 0
        for p in params:
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        self.buf = torch.zeros(off, dtype=dtype, device=device)
        self.ready = 0
        self.got = [False] * len(params)
        self.work = None
        self.launched = False


class DistributedDataParallel(nn.Module):
    def __init__(
        self,
        module: nn.Module,
        process_group=None,
        bucket_cap_mb: Optional[float] = None,
        first_bucket_mb: float = 4.0,
        broadcast_buffers: bool = True,
        comm_dtype: Optional[torch.dtype] = torch.float32,
        device_ids=None,  # accepted for API compatibility with torch DDP
        find_unused_parameters: bool = False,
        comm=None,
        buckets_at_world_1: bool = False,
    ):
        """``comm_dtype``: gradient bucket / all-reduce dtype (fp32 default; ``None`` = each
        parameter's dtype).  ``buckets_at_world_1``: build the bucket machinery even for a single
        rank (tests of the bucket / deferred-all-reduce / graph paths on a one-GPU box).
        ``bucket_cap_mb=None``: the all-reduce saturation point of a measured busbw sweep for this
        world size (``parallel/tuning.py``), 64 MiB without one."""
        super().__init__()
        if bucket_cap_mb is None:
            from .tuning import bucket_mb

            w = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
            bucket_cap_mb = bucket_mb(w)
        self.bucket_cap_mb = float(bucket_cap_mb)
        self.module = module
        self.process_group = process_group
        # bucket all-reduces go through the comm layer: Hyperion's native RCCL communicator (own
        # high-priority stream) on GPU, torch.distributed elsewhere (parallel/comm.py)
        dev = next((p.device for p in module.parameters()), torch.device("cpu"))
        self.comm = comm if comm is not None else (get_comm(dev, process_group) if dist.is_available()
                                                   and dist.is_initialized() else None)
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self._sync = True
        self.defer_allreduce = False
        # set while the first of a two-part backward runs (top stages; see TrainStep's split
        # graphs): the end-of-backward callback then keeps the bucket state for the second part
        self.partial_backward = False
        self._buckets: List[_Bucket] = []
        self._where: Dict[nn.Parameter, Tuple[_Bucket, int]] = {}
        self._next_launch = 0
        self._callback_queued = False
        self._hooks = []
        from ..ops.multi_tensor import TableCache

        self._tables = TableCache()  # multi-tensor pack tables, one per bucket and dtype pair
        if self.world > 1 or (buckets_at_world_1 and self.comm is not None):
            if self.world > 1:
                _flat_broadcast([p.data for p in module.parameters()] + list(module.buffers()), 0, process_group)
            self._build_buckets(bucket_cap_mb, first_bucket_mb, comm_dtype)
            for p in module.parameters():
                if p.requires_grad:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._grad_ready))

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self, cap_mb: float, first_mb: float, comm_dtype: Optional[torch.dtype]) -> None:
        params = [p for p in self.module.parameters() if p.requires_grad]
        params.reverse()  # gradients become ready roughly in reverse registration order
        # a bucket never straddles a graph-stage cut (models with graph_stage_modules(): the
        # split hipGraph step reduces the top stage's buckets while the bottom's backward runs)
        stage_of: Dict[int, int] = {}
        fn = getattr(self.module, "graph_stage_modules", None)
        if callable(fn):
            for si, mods in enumerate(fn()):
                for mod in mods:
                    for p in mod.parameters():
                        stage_of[id(p)] = si
        groups: List[Tuple[torch.dtype, torch.device, List[nn.Parameter]]] = []
        cur: List[nn.Parameter] = []
        cur_bytes = 0
        cur_key = None
        limit = first_mb * 2**20
        for p in params:
            dt = comm_dtype if (comm_dtype is not None and p.is_floating_point()) else p.dtype
            key = (dt, p.device, stage_of.get(id(p), -1))
            nbytes = p.numel() * torch.empty((), dtype=dt).element_size()
            if cur and (key != cur_key or cur_bytes + nbytes > limit):
                groups.append((cur_key[0], cur_key[1], cur))
                cur, cur_bytes = [], 0
                limit = cap_mb * 2**20
            cur.append(p)
            cur_bytes += nbytes
            cur_key = key
        if cur:
            groups.append((cur_key[0], cur_key[1], cur))
        for i, (dt, dev, ps) in enumerate(groups):
            b = _Bucket(i, ps, dt, dev)
            self._buckets.append(b)
            for i, p in enumerate(ps):
                self._where[p] = (b, i)

    def bucket_sizes(self) -> List[int]:
        return [b.buf.numel() for b in self._buckets]

    # ------------------------------------------------------------------ hooks
    def _grad_ready(self, p: nn.Parameter) -> None:
        # (runs on the stream autograd gives the parameter's AccumulateGrad: the stream of the
        # forward op that consumed it — where the gradient was produced)
        if not self._sync or p.grad is None:
            return
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b, i = self._where[p]
        if b.got[i]:
            return
        b.got[i] = True
        b.ready += 1
        if b.ready == len(b.params):
            self._pack(b)
            if not self.defer_allreduce:
                self._launch_ready()

    def _pack(self, b: _Bucket) -> None:
        """Copy (+ up-convert) a complete bucket's gradients into its slots: one multi-tensor
        launch per (gradient dtype, bucket dtype) pair instead of one copy kernel per parameter.
        Gradients wait in ``p.grad`` until their bucket is complete; a deferred weight-gradient
        reduce (or a parked weight gradient, ops/conv.py) may still owe the LAST of them its values,
        so the one flush happens here, before the pack reads them."""
        _flush_wgrad()
        dev = b.buf.device
        if b.buf.is_cuda:
            _streams.join(dev)  # gradients produced on the weight-gradient side stream
        groups: Dict[Tuple[torch.dtype, torch.dtype], Tuple[List[torch.Tensor], List[torch.Tensor]]] = {}
        with torch.no_grad():
            for i, p in enumerate(b.params):
                g = p.grad
                if g is None or not b.got[i]:  # an unused parameter: _finalize zero-fills its slot
                    continue
                off, n = b.offsets[i], p.numel()
                slot = _param_view(b.buf[off : off + n], p)
                if g.data_ptr() == slot.data_ptr():  # AccumulateGrad already summed into the slot
                    continue
                if (b.buf.is_cuda and _mt_ok(g, slot)):
                    srcs, dsts = groups.setdefault((g.dtype, slot.dtype), ([], []))
                    srcs.append(g)
                    dsts.append(slot)
                else:
                    slot.copy_(g)  # pack (+ up-convert into an fp32 bucket); the all-reduce averages
            for (sdt, ddt), (srcs, dsts) in groups.items():
                tab = self._tables.get(f"pack{b.index}_{sdt}_{ddt}", [srcs, dsts])
                from ..ops import _native

                _native.native().copy_mt(tab.ptrs, tab.sizes, tab.blocks, tab.T, tab.chunk,
                                         _native.DTYPE_CODE[sdt], _native.DTYPE_CODE[ddt])
            for p in b.params:
                if p.grad is not None and b.buf.dtype != p.dtype:
                    p.grad = None  # consumed: the optimizer reads p.main_grad; the next backward steals

    def _launch_ready(self) -> None:
        while self._next_launch < len(self._buckets):
            b = self._buckets[self._next_launch]
            if b.ready < len(b.params):
                break
            if b.buf.is_cuda:
                _streams.join(b.buf.device)  # packs issued on the weight-gradient side stream
            # under a segmented hipGraph capture (train/segments.py) the all-reduce is an eager hole
            # between two graph segments: every replay re-issues it right where this bucket became
            # complete, so it overlaps the rest of the captured backward
            _segments.eager(lambda b=b: self._issue(b))
            b.launched = True
            self._next_launch += 1

    def _issue(self, b: _Bucket) -> None:
        range_push(f"ddp_allreduce_b{b.index}")
        b.work = self.comm.all_reduce(b.buf, "avg")
        range_pop()

    @staticmethod
    def _wait(b: _Bucket) -> None:
        if b.work is not None:
            b.work.wait()  # stream-ordered: the compute stream waits on RCCL, the host does not
            b.work = None

    def _finalize(self) -> None:
        if self.partial_backward:  # more of this step's backward follows: keep the bucket state
            self._callback_queued = False
            return
        # parameters that got no gradient this step contribute zeros (find_unused_parameters)
        for b in self._buckets[self._next_launch :]:
            if b.ready < len(b.params):
                self._pack(b)  # the gradients that did arrive
                with torch.no_grad():
                    for i, (p, off) in enumerate(zip(b.params, b.offsets)):
                        if not b.got[i]:
                            b.buf[off : off + p.numel()].zero_()
                            b.got[i] = True
                b.ready = len(b.params)
        if not self.defer_allreduce:
            self._launch_ready()
        for b in self._buckets:
            if b.launched:
                _segments.eager(lambda b=b: self._wait(b))
            for p, off in zip(b.params, b.offsets):
                view = _param_view(b.buf[off : off + p.numel()], p)
                if view.dtype == p.dtype:
                    p.grad = view
                else:
                    p.grad = None
                    p.main_grad = view  # fp32 reduced gradient of a low-precision parameter
            b.ready = 0
            b.got = [False] * len(b.params)
            b.launched = False
        self._next_launch = 0
        self._callback_queued = False

    def complete_buckets(self) -> List[int]:
        """Indices of the buckets whose every gradient has been packed so far this step."""
        return [b.index for b in self._buckets if b.ready == len(b.params)]

    def allreduce_buckets(self, indices: Optional[List[int]] = None, wait: bool = True) -> list:
        """Reduce the given buckets (default: all) now (``defer_allreduce`` mode).

        The gradients already point at their bucket slices, so after this (an RCCL ``avg``) the
        optimizer reads the averaged gradients in place.  ``wait=False`` returns the work
        handles instead of ordering the current stream after them, so compute issued next (the
        second half of a split backward) overlaps the collectives on the comm stream; every rank
        must pass the same ``indices`` in the same order."""
        if not self._buckets or not self._sync:
            return []
        if self._buckets[0].buf.is_cuda:
            _streams.join(self._buckets[0].buf.device)
        works = []
        for b in self._buckets if indices is None else [self._buckets[i] for i in indices]:
            range_push(f"ddp_allreduce_b{b.index}")
            works.append(self.comm.all_reduce(b.buf, "avg"))
            range_pop()
        if wait:
            for w in works:
                if w is not None:
                    w.wait()
            return []
        return [w for w in works if w is not None]

    @property
    def bucketed(self) -> bool:
        return bool(self._buckets)

    # ------------------------------------------------------------------ module API
    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (no all-reduce) inside this context."""
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def sync_buffers(self) -> None:
        """Rank 0's buffers (BN running statistics) to every rank, in place (K5)."""
        bufs = [b for b in self.module.buffers() if b.numel() > 0]
        if bufs:
            _flat_broadcast(bufs, 0, self.process_group)

    def has_buffers(self) -> bool:
        return any(b.numel() > 0 for b in self.module.buffers())

    def forward(self, *args, **kwargs):
        if self.world > 1 and self.broadcast_buffers and self.has_buffers():
            # per-forward broadcast (torch DDP's broadcast_buffers=True); an eager hole when the
            # step is being captured as segments, so replays broadcast before every forward too
            _segments.eager(self.sync_buffers)
        return self.module(*args, **kwargs)

    def state_dict(self, *args, **kwargs):  # keep reference checkpoint keys (model.module.state_dict())
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True):
        return self.module.load_state_dict(state_dict, strict=strict)


DDP = DistributedDataParallel
