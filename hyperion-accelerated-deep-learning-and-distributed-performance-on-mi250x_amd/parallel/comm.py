"""Communication layer: one interface, two backends.

* ``NativeComm`` — Hyperion's C++ RCCL communicator (``csrc/comm/rccl_comm.cpp``): a raw
  ncclComm_t on its own highest-priority HIP stream, stream-ordered collectives fenced with
  hipEvents (the host never blocks), bootstrapped through the torchrun TCPStore.
* ``TorchComm`` — ``torch.distributed`` (RCCL via ProcessGroupNCCL on GPU, gloo on CPU): the CPU
  test path and the fallback.

Both return work handles whose ``wait()`` orders the caller's current stream after the
collective.

Failure handling (the reference's process-group timeout, ``distributed_utils.py:106-111``):
``NativeComm`` is created nonblocking and supervised by a watchdog thread
(``csrc/comm/watchdog.h``): a collective that misses ``timeout_s`` (default: the ``setup()``
timeout) or an RCCL async error aborts the communicator, and the next collective / ``wait()``
raises ``RuntimeError`` naming the collective.  ``HYPERION_COMM_ON_TIMEOUT=exit`` terminates the
rank instead (exit status 75) so ``torchrun --max-restarts`` can restart the job.  ``get_comm()`` picks native on GPU when the extension is loaded
(``HYPERION_COMM=torch`` forces the torch backend).  Reference: all collectives went through
ProcessGroupNCCL.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _native

_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "avg": dist.ReduceOp.AVG}


class _Done:
    def wait(self):
        return None

    def synchronize(self):
        return None

    def is_completed(self):
        return True


class _ScaleAfter:
    """A SUM collective's work handle whose wait() also divides the result by the world size (the
    "avg" of a reduction, in the caller's stream order after the collective)."""

    def __init__(self, work, t: torch.Tensor, world: int):
        self.work, self.t, self.world = work, t, world

    def wait(self):
        self.work.wait()
        self.t.div_(self.world)
        return True

    def is_completed(self):
        return self.work.is_completed()


class TorchComm:
    backend = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        if self.world == 1:
            return _Done()
        if op == "avg":  # SUM + 1/world: never ReduceOp.AVG (RCCL's ncclAvg drops output tails, rccl_comm.cpp)
            return _ScaleAfter(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True), t, self.world)
        return dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=True)

    def all_reduce_coalesced(self, ts: List[torch.Tensor], op: str = "sum"):
        works = [self.all_reduce(t, op) for t in ts]
        return works[-1] if works else _Done()

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum"):
        if self.world == 1:
            out.copy_(inp)
            return _Done()
        if op == "avg":
            w = dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            return _ScaleAfter(w, out, self.world)
        return dist.reduce_scatter_tensor(out, inp, op=_OPS[op], group=self.group, async_op=True)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        if self.world == 1:
            out.copy_(inp)
            return _Done()
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)

    def broadcast(self, t: torch.Tensor, root: int = 0):
        if self.world == 1:
            return _Done()
        return dist.broadcast(t, src=root, group=self.group, async_op=True)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor):
        if self.world == 1:
            out.copy_(inp)
            return _Done()
        return dist.all_to_all_single(out, inp, group=self.group, async_op=True)

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.group)


def group_key(group=None) -> str:
    """Stable name of a process group from its member ranks (global rank ids)."""
    if not dist.is_initialized():
        return "local"
    if group is None or group is dist.group.WORLD:
        return f"world{dist.get_world_size()}"
    ranks = dist.get_process_group_ranks(group)
    return "g" + "-".join(str(r) for r in ranks)


def default_timeout_s() -> float:
    """The communicator deadline: ``HYPERION_COMM_TIMEOUT_S``, else the ``setup()`` timeout."""
    env = os.environ.get("HYPERION_COMM_TIMEOUT_S")
    if env:
        return float(env)
    from .launch import current_timeout_s
    return current_timeout_s()


class NativeComm:
    """Hyperion C++ RCCL communicator bootstrapped over the default TCPStore.

    Bootstrap keys are per process group (``group_key``) and count communicators per group, so
    ranks that build communicators for different groups in different orders never read each
    other's ``ncclUniqueId`` (every member of ONE group must still create that group's
    communicators in the same order — the usual collective-call contract).
    """

    backend = "native"
    _per_group: dict = {}

    def __init__(self, device: torch.device, group=None, tag: Optional[str] = None,
                 timeout_s: Optional[float] = None):
        C = _native.native()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        gk = group_key(group)
        n = NativeComm._per_group.get(gk, 0) + 1
        NativeComm._per_group[gk] = n
        key = f"hyperion_rccl_uid/{gk}/{tag or n}"
        store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            store.set(key, C.rccl_unique_id())
        uid = store.get(key)
        self.timeout_s = float(timeout_s if timeout_s is not None else default_timeout_s())
        self._device = torch.device(device)
        self._seq = 0
        self._global_rank = dist.get_rank()
        self._c = C.RcclComm(bytes(uid), self.rank, self.world, self._device.index or 0, self.timeout_s)

    @property
    def stream_handle(self) -> int:
        return self._c.stream_handle

    def _issue(self, fn, *args):
        # HYPERION_FAULT=rank:seq:stall (utils/fault.py): stall THIS rank's comm stream on the GPU
        # ahead of its seq-th collective, so the collective misses its deadline (watchdog tests)
        self._seq += 1
        from ..utils.fault import comm_stall_s
        stall = comm_stall_s(self._global_rank, self._seq)
        if stall:
            s = torch.cuda.ExternalStream(self.stream_handle, device=self._device)
            with torch.cuda.stream(s):
                torch.cuda._sleep(int(stall * 2.0e9))  # ~clock cycles at ~2 GHz
        return fn(*args)

    def all_reduce(self, t, op="sum"):
        return self._issue(self._c.all_reduce, t, op)

    def all_reduce_coalesced(self, ts, op="sum"):
        return self._issue(self._c.all_reduce_coalesced, list(ts), op)

    def reduce_scatter(self, out, inp, op="sum"):
        return self._issue(self._c.reduce_scatter, out, inp, op)

    def all_gather(self, out, inp):
        return self._issue(self._c.all_gather, out, inp)

    def broadcast(self, t, root=0):
        return self._issue(self._c.broadcast, t, root)

    def all_to_all(self, out, inp):
        return self._issue(self._c.all_to_all, out, inp)

    def error(self) -> str:
        """'' while healthy, else why the watchdog failed the communicator."""
        return self._c.error()

    def abort(self) -> None:
        self._c.abort()

    def barrier(self) -> None:
        self._c.barrier()

    def async_error(self) -> str:
        return self._c.async_error()

    def destroy(self) -> None:
        self._c.destroy()


def get_comm(device: Optional[torch.device] = None, group=None):
    """Native RCCL communicator on GPU (extension loaded, world > 1), else torch.distributed."""
    want = os.environ.get("HYPERION_COMM", "native").lower()
    if (want == "native" and device is not None and torch.device(device).type == "cuda" and dist.is_initialized()
            and dist.get_world_size(group) > 1 and _native.available()):
        return NativeComm(device, group)
    return TorchComm(group)
