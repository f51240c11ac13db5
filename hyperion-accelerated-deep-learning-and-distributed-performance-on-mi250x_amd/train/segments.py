"""Segmented hipGraph capture: a training step recorded as graphs with eager "holes".

Reference context: the reference's FSDP trainers run every step eagerly under torch FSDP, one
Python hook per unit per phase (``02_development/distributed_utils.py:318-354, 477-524``; SURVEY
C25/C26, §2.2 FSDP).  A Hyperion FSDP step cannot be ONE graph: its all-gathers and
reduce-scatters are eager RCCL (or gloo) calls issued from autograd hooks, and recording RCCL into a
graph is not what the multi-rank tests can exercise.  Instead the step is captured ONCE as a list of
segments: every time the step is about to issue (or wait for) a collective, the current capture
ends, the collective runs for real and is appended to the schedule as an eager action, and a new
capture begins.  Replaying the step = replay segment 0, run action 0, replay segment 1, ... — the
~10^3 kernels of the step cost a few dozen graph launches, and every collective still overlaps
the compute segments between its issue and its wait (issue and wait are separate actions).

All segments share one memory pool, so a tensor produced in segment i and consumed in segment j
keeps its address on every replay; the actions must only touch persistent buffers (FSDP's
``persistent`` mode keeps the full-parameter and gradient buffers allocated for exactly this).
"""
from __future__ import annotations

import os
import time
import warnings
from typing import Callable, List, Optional

import torch

_ACTIVE: Optional["SegmentedGraph"] = None
_PROFILE = os.environ.get("HYPERION_SEG_PROFILE") == "1"


def _capture_is_empty() -> bool:
    """Nothing recorded yet by the capture on the current stream (native query; False if unknown)."""
    try:
        from ..ops import _native

        if not _native.available():
            return False
        return bool(_native.native().capture_is_empty(torch.cuda.current_stream().cuda_stream))
    except Exception:  # noqa: BLE001 - an unknown answer keeps the segment
        return False


def active() -> Optional["SegmentedGraph"]:
    """The capture in progress, if any (collective call sites route through :func:`eager`)."""
    return _ACTIVE


def eager(fn: Callable[[], object]):
    """Run ``fn`` now; under a segmented capture, as an eager action between two segments."""
    seg = _ACTIVE
    if seg is None:
        return fn()
    return seg.hole(fn)


class SegmentedGraph:
    """Capture ``body()`` as graph segments split at :func:`eager` calls; ``replay()`` re-runs it."""

    def __init__(self):
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.actions: List[Callable[[], object]] = []  # actions[i] runs after graphs[i]
        # empty[i]: segment i recorded no work (two holes back to back, e.g. one unit's gather wait
        # and the next unit's gather issue): never replayed, so the holes run as one action
        self.empty: List[bool] = []
        self.host_s: dict = {}
        self.stream: Optional[torch.cuda.Stream] = None
        self._pool = None
        self.out = None

    # -- capture ----------------------------------------------------------------------------
    def _begin(self) -> None:
        g = torch.cuda.CUDAGraph()
        if self._pool is None:
            # a fresh handle up front: CUDAGraph.pool() is only valid after a finished capture
            self._pool = torch.cuda.graph_pool_handle()
        self.graphs.append(g)
        # relaxed error mode: the holes' collectives may run helper threads (gloo's async work copies
        # GPU tensors from its own thread) whose runtime calls must not invalidate the capture, and a
        # hole inside backward ends / begins a segment on the autograd engine's thread, which a
        # thread-local capture forbids
        g.capture_begin(pool=self._pool, capture_error_mode="relaxed")

    def _end(self) -> None:
        empty = _capture_is_empty()
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # "The CUDA Graph is empty": expected, never replayed
            self.graphs[-1].capture_end()
        self.empty.append(empty)

    def hole(self, fn: Callable[[], object]):
        """End the current segment, run ``fn`` eagerly (recorded), start the next segment."""
        self._end()
        res = fn()
        self.actions.append(fn)
        self._begin()
        return res

    def capture(self, body: Callable[[], object]):
        global _ACTIVE
        assert _ACTIVE is None, "nested segmented capture"
        self.stream = torch.cuda.Stream()
        self.stream.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        with torch.cuda.stream(self.stream):
            _ACTIVE = self
            try:
                self._begin()
                self.out = body()
                self._end()
            except BaseException:
                # close a capture the body left open, so the failure surfaces as this exception and
                # not as a terminate() from the graph's destructor
                if torch.cuda.is_current_stream_capturing():
                    try:
                        self.graphs[-1].capture_end()
                    except Exception:
                        pass
                self.graphs.clear()
                self.empty.clear()
                raise
            finally:
                _ACTIVE = None
        torch.cuda.current_stream().wait_stream(self.stream)
        torch.cuda.synchronize()
        return self.out

    # -- replay -----------------------------------------------------------------------------
    def replay(self):
        s = self.stream
        s.wait_stream(torch.cuda.current_stream())
        prof = _PROFILE
        with torch.cuda.stream(s):
            for i, g in enumerate(self.graphs):
                t0 = time.perf_counter() if prof else 0.0
                if not self.empty[i]:
                    g.replay()
                if prof:
                    t1 = time.perf_counter()
                    self.host_s[("graph", i)] = self.host_s.get(("graph", i), 0.0) + t1 - t0
                if i < len(self.actions):
                    self.actions[i]()
                    if prof:
                        self.host_s[("hole", i)] = self.host_s.get(("hole", i), 0.0) + time.perf_counter() - t1
        torch.cuda.current_stream().wait_stream(s)
        return self.out

    def host_profile(self) -> dict:
        """HYPERION_SEG_PROFILE=1: host seconds spent per graph replay / hole action, summed over replays."""
        return {f"{k}{i}": round(v, 6) for (k, i), v in sorted(self.host_s.items(), key=lambda kv: -kv[1])}

    @property
    def num_segments(self) -> int:
        """Graph segments replayed per step (empty ones are skipped)."""
        return sum(1 for e in self.empty if not e)

    @property
    def num_holes(self) -> int:
        return len(self.actions)


class SegmentedStep:
    """``step()`` = ``fn()`` captured as segments after ``warmup`` eager calls (GraphedClosure's
    contract: ``fn`` zeroes grads in place or lets the captured backward steal fresh ones, reads
    persistent inputs, returns a tensor)."""

    def __init__(self, fn: Callable[[], torch.Tensor], warmup: int = 3, module: Optional[torch.nn.Module] = None):
        self.fn = fn
        self.warmup = warmup
        self.module = module
        self.seg: Optional[SegmentedGraph] = None
        self._counters = None

    def __call__(self) -> torch.Tensor:
        if self.seg is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(self.warmup):
                    self.fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            from ..ops.multi_tensor import flush_pending

            from ..ops.batchnorm import HostCounterReplay

            counters = None
            if self.module is not None:
                for p in self.module.parameters():
                    p.grad = None
                counters = HostCounterReplay(self.module)
            seg = SegmentedGraph()
            try:
                seg.capture(self.fn)
            finally:
                flush_pending()
            self.seg = seg
            self._counters = counters.captured() if counters is not None else None
        out = self.seg.replay()
        if self._counters is not None:
            self._counters.replayed()  # BN num_batches_tracked mirrors advance once per replayed step
        return out
