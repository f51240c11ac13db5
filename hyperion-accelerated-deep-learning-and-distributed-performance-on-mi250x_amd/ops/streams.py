"""Weight-gradient side stream.

Nothing in the backward pass consumes a weight gradient — only the optimizer (or the gradient
buckets of data parallelism) does, after the backward.  On MI355X the ResNet-50 backward is a
chain of latency-bound, under-filled launches (per-layer data gradient -> BN backward -> data
gradient ..., 10-25 us each at 0.1-0.3 of the chip's MFMA rate), so the weight-gradient GEMMs
(``conv_wgrad.hip`` and its split-K reduce, ~1.5 ms of a 6.2 ms step) run on a second HIP stream,
concurrently with that chain, filling the CUs it leaves idle.  hipGraph capture records the fork
(``side.wait_stream(current)``) and the join as graph edges, so replays overlap the same way.

Rules that keep it correct:
* inputs are ``record_stream``-ed on the side stream and the output on the current stream (the
  caching allocator then never recycles a block one stream still reads);
* the side stream is joined into the current stream at the end of every backward pass (an
  autograd-engine callback queued at the first side launch), so optimizers and any code after
  ``backward()`` see finished gradients;
* consumers INSIDE the backward (gradient-bucket hooks) call :func:`join` first, or do their own
  work on the side stream (:func:`side_of`);
* only used when AccumulateGrad will steal the gradient (``param.grad is None``): an accumulate
  into an existing ``.grad`` would read it on the current stream too early.

Reference counterpart: none — the reference left all of backward to MIOpen/rocBLAS on one stream
(SURVEY §2.4 conv row).

Measured on MI355X (ResNet-50 bf16 batch 32, hipGraph step): the wgrad kernels do overlap the
chain (summed kernel time 7.40 ms over a 6.77 ms span) but every kernel slows down by as much —
6.23 ms/step with the side stream vs 6.21 without — so it is OFF by default
(``HYPERION_WGRAD_STREAM=1`` enables it; profiles/r02).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable, Optional

import torch

_SIDE: Dict[int, "torch.cuda.Stream"] = {}
_PENDING: set = set()


def enabled() -> bool:
    return os.environ.get("HYPERION_WGRAD_STREAM", "0") == "1"


def side_stream(device: torch.device) -> "torch.cuda.Stream":
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    s = _SIDE.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _SIDE[idx] = s
    return s


def join(device: Optional[torch.device] = None) -> None:
    """Order the current stream after everything issued so far on the side stream."""
    idxs = list(_PENDING) if device is None else [torch.device(device).index or 0]
    for i in idxs:
        if i in _PENDING:
            torch.cuda.current_stream(i).wait_stream(_SIDE[i])
            _PENDING.discard(i)


def pending(device: torch.device) -> bool:
    return (torch.device(device).index or 0) in _PENDING


def run_on_side(fn: Callable[[], torch.Tensor], inputs: Iterable[torch.Tensor], device: torch.device) -> torch.Tensor:
    """Run ``fn`` (which launches kernels and returns a tensor) on the side stream."""
    cur = torch.cuda.current_stream(device)
    side = side_stream(device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        out = fn()
    for t in inputs:
        if t is not None and t.is_cuda:
            t.record_stream(side)
    out.record_stream(cur)
    idx = side.device.index
    if idx not in _PENDING:
        _PENDING.add(idx)
        try:  # join at the end of this backward pass
            torch.autograd.Variable._execution_engine.queue_callback(lambda: join())
        except RuntimeError:  # not inside a backward pass: join now
            join()
    return out


def use_side_for(param: torch.Tensor) -> bool:
    """The side stream may produce ``param``'s gradient (it will be stolen, not accumulated)."""
    return enabled() and param.is_cuda and param.grad is None


def on_stream(s: Optional["torch.cuda.Stream"]):
    """Context that makes s current (no-op when s is None or already current).  Autograd
    hooks run on the engine's thread with the current stream of the node that fired them — for a
    leaf's AccumulateGrad not necessarily the stream the step runs on — so data-parallel wrappers
    re-enter the forward's stream before they copy gradients or issue collectives."""
    import contextlib

    if s is None or s == torch.cuda.current_stream(s.device):
        return contextlib.nullcontext()
    return torch.cuda.stream(s)
