"""Training-step engine: eager or hipGraph-captured (fwd + bwd + optimizer as one graph).

The reference amortized launch overhead with ``torch.compile(mode="reduce-overhead")`` /
Inductor (``compilation_optimization.py:96-103``, C32).  Hyperion has no tracing compiler: the
static-shape step is captured once into a hipGraph and replayed, so a ResNet-50 step (≈1,000
kernels: convs, fused BN, fused optimizer) costs one graph launch on the host.

Requirements for capture (all satisfied by Hyperion ops): no host syncs inside the step, no
pageable H2D copies, device-side optimizer scalars (``FusedAdam`` keeps step count on device).

Data-parallel steps (Hyperion ``DDP`` over more than one rank, ``broadcast_buffers=False``) are
captured as TWO graphs — forward+backward (the gradient hooks pack the buckets) and the optimizer
— with the bucket all-reduces issued eagerly between the replays (``DDP.defer_allreduce``): no
RCCL call is ever recorded into a graph, and the ~500 per-step kernel launches still cost two
graph launches.

When the model exposes ``graph_stages()`` (``[bottom, top]`` with ``forward == top∘bottom``;
ResNet splits after layer1), the backward itself is cut in two graphs at that boundary: graph 1 =
forward + backward of the top (its buckets — ~85% of ResNet-50's gradient bytes — are complete),
then those buckets' all-reduces are issued on the comm stream WITHOUT ordering the compute
stream after them, graph 2 = backward of the bottom (overlapping the collectives), the remaining
buckets are reduced, and graph 3 = the optimizer after all collectives.  On point-to-point xGMI a
2-GPU all-reduce of ResNet-50's 102 MB of fp32 gradient buckets runs over ONE ≈64-77 GB/s link: hiding it
behind the bottom half's backward is worth ~10% of a 7 ms step.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Optional

import torch
import torch.nn as nn



def autocast_ctx(device: torch.device, dtype: Optional[torch.dtype]):
    if dtype is None or dtype == torch.float32:
        return contextlib.nullcontext()
    return torch.autocast(device_type=device.type, dtype=dtype)



def _has_dropout(module: torch.nn.Module) -> bool:
    """Any active dropout (nn.Dropout-family modules, or an attention module's dropout rate)."""
    for m in module.modules():
        if isinstance(m, torch.nn.modules.dropout._DropoutNd) and m.p > 0:
            return True
        for attr in ("dropout_p", "attn_dropout", "dropout"):
            v = getattr(m, attr, None)
            if isinstance(v, float) and v > 0:
                return True
    return False

class TrainStep:
    """``loss = step(x, y)``; captures a hipGraph on GPU when ``graph=True``."""

    def __init__(
        self,
        model: nn.Module,
        optimizer: torch.optim.Optimizer,
        loss_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
        amp_dtype: Optional[torch.dtype] = torch.bfloat16,
        graph: bool = False,
        warmup_iters: int = 3,
        scaler=None,
        split_backward: bool = True,
        ddp_schedule: str = "segmented",
    ):
        """``ddp_schedule`` (a bucketed Hyperion DDP model, graph mode): ``"segmented"`` (default;
        ``"auto"`` is an alias) = the whole step captured as segments with every bucket's
        all-reduce issue and wait as eager holes (``train/segments.py``): each bucket overlaps the
        rest of the captured backward, at the cost of one graph launch per hole (ResNet-50 at world
        1 with the native RCCL communicator: 5.13 ms vs 4.58 plain, profiles/r05/ddp_schedule_ab.json);
        ``"graph"`` = ONE graph with the bucket all-reduces recorded into it (the native RCCL
        communicator's comm stream forked from and joined into the capture: no host holes at all);
        ``"split3"`` = A/B only, three graphs (top forward+backward | bottom backward overlapping
        the top buckets' all-reduce | optimizer) when the model exposes ``graph_stages``, else two
        graphs around the all-reduces — measured 14.5 ms/step at world 1, 3x the plain step, so it
        is never picked by default."""
        if ddp_schedule == "auto":
            ddp_schedule = "segmented"
        if ddp_schedule not in ("split3", "segmented", "graph"):
            raise ValueError(f"ddp_schedule {ddp_schedule!r}")
        self.ddp_schedule = ddp_schedule
        self.seg = None
        self.model = model
        self.opt = optimizer
        self.loss_fn = loss_fn
        self.amp_dtype = amp_dtype
        self.use_graph = graph and torch.cuda.is_available()
        self.warmup_iters = warmup_iters
        self.scaler = scaler
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_x: Optional[torch.Tensor] = None
        self.static_y: Optional[torch.Tensor] = None
        self.static_loss: Optional[torch.Tensor] = None
        self.graph2: Optional[torch.cuda.CUDAGraph] = None
        self.graph3: Optional[torch.cuda.CUDAGraph] = None
        self.split_backward = split_backward
        self._phase1: list = []
        self._phase2: list = []
        self._keep = None
        self._counters = None  # BatchNormAct2d num_batches_tracked mirrors under replay

    def _ddp(self):
        """The model if it is a bucketed Hyperion DDP whose step can be split around its collectives."""
        from ..parallel.ddp import DistributedDataParallel

        m = self.model
        if isinstance(m, DistributedDataParallel) and m.bucketed and not m.broadcast_buffers and self.scaler is None:
            return m
        return None

    def _stages(self):
        """``[bottom, top]`` of a DDP-wrapped model that can split its backward, else None."""
        ddp = self._ddp()
        if ddp is None or not self.split_backward:
            return None
        fn = getattr(ddp.module, "graph_stages", None)
        st = fn() if callable(fn) else None
        if st is None or len(st) != 2:
            return None
        # a dropout mask is regenerated in backward from the generator offset that each graph
        # replay rewrites: forward in graph 1 and the bottom backward in graph 2 would see different
        # masks — a bottom stage with active dropout keeps the single-graph step
        bottom = st[0] if isinstance(st[0], torch.nn.Module) else ddp.module  # (a callable: the whole model)
        if _has_dropout(bottom):
            return None
        return st

    def _loss_in(self, out: torch.Tensor) -> torch.Tensor:
        """The logits as the loss takes them: fp32, unless the loss fuses the cast itself."""
        if out.dtype == torch.float32 or getattr(self.loss_fn, "accepts_low_precision", False):
            return out
        return out.float()

    def _fwd_bwd_top(self, x: torch.Tensor, y: torch.Tensor, stages, zero_in_place: bool = False):
        """Forward through both stages, backward through the top one only."""
        if zero_in_place:
            self.opt.zero_grad(set_to_none=False)
        ddp = self._ddp()
        with autocast_ctx(x.device, self.amp_dtype):
            h = stages[0](x)
            h2 = h.detach().requires_grad_(True)
            out = stages[1](h2)
            loss = self.loss_fn(self._loss_in(out), y)
        ddp.partial_backward = True
        try:
            loss.backward()
        finally:
            ddp.partial_backward = False
        return loss.detach(), h, h2

    def split_step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Eager two-part backward with the top buckets' all-reduce overlapping the bottom
        backward (the captured path's schedule without graphs; CPU-testable over gloo)."""
        stages = self._stages()
        ddp = self._ddp()
        assert stages is not None and ddp is not None and ddp.defer_allreduce
        self.opt.zero_grad(set_to_none=False)
        loss, h, h2 = self._fwd_bwd_top(x, y, stages)
        first = ddp.complete_buckets()
        works = ddp.allreduce_buckets(first, wait=False)
        h.backward(h2.grad)
        works += ddp.allreduce_buckets([i for i in range(len(ddp.bucket_sizes())) if i not in first], wait=False)
        for w in works:
            w.wait()
        self.opt.step()
        return loss

    def _fwd_bwd(self, x: torch.Tensor, y: torch.Tensor, zero_in_place: bool = False) -> torch.Tensor:
        if zero_in_place:  # graph mode: gradients keep their addresses, zeroed in place
            self.opt.zero_grad(set_to_none=False)
        dev = x.device
        with autocast_ctx(dev, self.amp_dtype):
            out = self.model(x)
            loss = self.loss_fn(self._loss_in(out), y)
        loss.backward()
        return loss.detach()

    def _body(self, x: torch.Tensor, y: torch.Tensor, zero_in_place: bool = False) -> torch.Tensor:
        if self.scaler is not None:
            if zero_in_place:
                self.opt.zero_grad(set_to_none=False)
            with autocast_ctx(x.device, self.amp_dtype):
                out = self.model(x)
                loss = self.loss_fn(self._loss_in(out), y)
            self.scaler.scale(loss).backward()
            self.scaler.step(self.opt)
            self.scaler.update()
            return loss.detach()
        loss = self._fwd_bwd(x, y, zero_in_place)
        ddp = self._ddp()
        if ddp is not None and ddp.defer_allreduce:
            ddp.allreduce_buckets()
        self.opt.step()
        return loss

    def eager_step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        self.opt.zero_grad(set_to_none=True)
        return self._body(x, y)

    def _capture(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """Warm up on a side stream, then capture one step.

        The gradients are released right before the capture, so inside it autograd STEALS each
        fresh weight gradient (an allocation of the graph's private pool, at the same address on
        every replay) instead of adding it into a kept ``.grad`` buffer — that add was one extra
        kernel per parameter per step (161 launches, ~0.77 ms of a ResNet-50 step).  The fused
        optimizer's tables, built during warm-up, are re-pointed at the captured gradients
        (``ops/multi_tensor.py``: deferred until the capture ends, ``flush_pending``).
        """
        self.static_x = x.clone()
        self.static_y = y.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.opt.zero_grad(set_to_none=True)
            for _ in range(self.warmup_iters):
                self._body(self.static_x, self.static_y, zero_in_place=True)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        from ..ops.batchnorm import HostCounterReplay

        from ..ops.multi_tensor import flush_pending

        counters = HostCounterReplay(self.model)
        zero_flag = getattr(self.opt, "zero_grad_in_step", None)
        if self.scaler is None:
            self.opt.zero_grad(set_to_none=True)
            if zero_flag:  # stolen gradients are rewritten by every replay: no zero pass needed
                self.opt.zero_grad_in_step = False
        try:
            self._capture_graphs()
        finally:
            self._counters = counters.captured()
            flush_pending()
            if zero_flag is not None:
                self.opt.zero_grad_in_step = zero_flag

    def _capture_graphs(self) -> None:
        ddp = self._ddp()
        if ddp is not None and self.ddp_schedule == "graph":
            ddp = None  # the single-graph capture below records the all-reduces too
        elif ddp is not None and self.ddp_schedule == "segmented":
            from .segments import SegmentedGraph

            seg = SegmentedGraph()
            self.static_loss = seg.capture(lambda: self._body(self.static_x, self.static_y))
            self.seg, self.graph = seg, seg.graphs[0]
            return
        stages = self._stages() if ddp is not None else None
        if ddp is not None and stages is not None:  # three graphs: top fwd+bwd | bottom bwd | optimizer
            g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                self.static_loss, h, h2 = self._fwd_bwd_top(self.static_x, self.static_y, stages)
            self._phase1 = ddp.complete_buckets()
            self._phase2 = [i for i in range(len(ddp.bucket_sizes())) if i not in self._phase1]
            with torch.cuda.graph(g2, pool=g1.pool()):
                h.backward(h2.grad)
            with torch.cuda.graph(g3, pool=g1.pool()):
                self.opt.step()
            torch.cuda.synchronize()
            self._keep = (h2,)
            self.graph, self.graph2, self.graph3 = g1, g2, g3
            return
        if ddp is not None:  # two graphs around the (eager) bucket all-reduces
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                self.static_loss = self._fwd_bwd(self.static_x, self.static_y)
            with torch.cuda.graph(g2, pool=g1.pool()):
                self.opt.step()
            torch.cuda.synchronize()
            self.graph, self.graph2 = g1, g2
            return
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            # with a loss scaler the grads stay allocated and are zeroed in place (its unscale
            # table is built in warm-up); otherwise they are stolen fresh (see _capture)
            self.static_loss = self._body(self.static_x, self.static_y, zero_in_place=self.scaler is not None)
        torch.cuda.synchronize()
        self.graph = g

    def __call__(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if not self.use_graph:
            return self.eager_step(x, y)
        if self.graph is None:
            ddp = self._ddp()
            if ddp is not None:
                # graph schedules: the all-reduces run between the graphs; segmented: from the
                # bucket hooks, as holes of the capture
                ddp.defer_allreduce = self.ddp_schedule == "split3"
            self._capture(x, y)
        if x.data_ptr() != self.static_x.data_ptr():
            self.static_x.copy_(x, non_blocking=True)
        if y.data_ptr() != self.static_y.data_ptr():
            self.static_y.copy_(y, non_blocking=True)
        if self.seg is not None:
            self.seg.replay()
            self._counters.replayed()
            return self.static_loss
        self.graph.replay()
        self._counters.replayed()
        if self.graph3 is not None:
            # top buckets reduce on the comm stream while the bottom backward replays
            works = self.model.allreduce_buckets(self._phase1, wait=False)
            self.graph2.replay()
            works += self.model.allreduce_buckets(self._phase2, wait=False)
            for w in works:
                w.wait()
            self.graph3.replay()
        elif self.graph2 is not None:
            self.model.allreduce_buckets()
            self.graph2.replay()
        return self.static_loss


class GraphedClosure:
    """Capture an arbitrary training-step closure into a hipGraph after ``warmup`` eager calls.

    ``fn`` must zero gradients IN PLACE (``zero_grad(set_to_none=False)``), read its inputs from
    persistent tensors and return a tensor (e.g. the loss); replays then re-run the whole step —
    forward, backward, clipping, optimizer — as one graph launch.  Used where the model call is not
    ``loss_fn(model(x), y)`` (Llama with masks and labels, the LM with its fused head).
    """

    def __init__(self, fn: Callable[[], torch.Tensor], warmup: int = 3, module: Optional[nn.Module] = None):
        """``module``: the model the closure trains (its BatchNormAct2d counters follow replays, and
        its gradients are released before capture so the captured backward steals fresh ones —
        ``fn`` must then not accumulate gradients across calls)."""
        self.fn = fn
        self.warmup = warmup
        self.module = module
        self.counters = None
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out: Optional[torch.Tensor] = None

    def __call__(self) -> torch.Tensor:
        if self.graph is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    self.fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            from ..ops.batchnorm import HostCounterReplay

            from ..ops.multi_tensor import flush_pending

            counters = HostCounterReplay(self.module) if self.module is not None else None
            if self.module is not None:
                # let autograd steal the captured step's fresh gradients (no per-parameter add into
                # kept buffers; the optimizer tables are re-pointed, see TrainStep._capture)
                for p in self.module.parameters():
                    p.grad = None
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    self.out = self.fn()
            finally:
                flush_pending()
            torch.cuda.synchronize()
            self.counters = counters.captured() if counters is not None else None
            self.graph = g
        self.graph.replay()
        if self.counters is not None:
            self.counters.replayed()
        return self.out
