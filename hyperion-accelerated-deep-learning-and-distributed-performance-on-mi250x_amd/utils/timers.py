"""Timers.

The reference times everything as ``torch.cuda.synchronize(); time.time()`` brackets
(SURVEY §5.1).  ``EventTimer`` uses hipEvents recorded on the current stream (device time, no
host jitter); ``WallTimer`` reproduces the reference method for apples-to-apples comparisons.
"""
from __future__ import annotations

import statistics
import time
from typing import List, Optional

import torch


def cuda_sync() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class WallTimer:
    """``synchronize(); time.perf_counter()`` bracket (reference methodology)."""

    def __init__(self, sync: bool = True):
        self.sync = sync
        self.t0 = 0.0
        self.elapsed = 0.0

    def __enter__(self):
        if self.sync:
            cuda_sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.sync:
            cuda_sync()
        self.elapsed = time.perf_counter() - self.t0
        return False


class EventTimer:
    """Accumulates hipEvent-timed intervals; falls back to wall time on CPU."""

    def __init__(self):
        self.samples_ms: List[float] = []
        self._start: Optional[torch.cuda.Event] = None
        self._t0 = 0.0

    def start(self) -> None:
        if torch.cuda.is_available():
            self._start = torch.cuda.Event(enable_timing=True)
            self._start.record()
        else:
            self._t0 = time.perf_counter()

    def stop(self) -> float:
        if torch.cuda.is_available() and self._start is not None:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            end.synchronize()
            ms = self._start.elapsed_time(end)
        else:
            ms = (time.perf_counter() - self._t0) * 1e3
        self.samples_ms.append(ms)
        return ms

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()
        return False

    @property
    def mean_ms(self) -> float:
        return statistics.fmean(self.samples_ms) if self.samples_ms else 0.0

    @property
    def median_ms(self) -> float:
        return statistics.median(self.samples_ms) if self.samples_ms else 0.0


def time_fn(fn, iters: int = 10, warmup: int = 3) -> float:
    """Median device ms of ``fn()`` over ``iters`` runs after ``warmup``."""
    for _ in range(warmup):
        fn()
    cuda_sync()
    t = EventTimer()
    for _ in range(iters):
        with t:
            fn()
    return t.median_ms
