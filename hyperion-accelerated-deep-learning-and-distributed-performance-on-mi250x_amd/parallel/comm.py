"""Communication layer: one interface, two backends.

* ``NativeComm`` — Hyperion's C++ RCCL communicator (``csrc/comm/rccl_comm.cpp``): a raw
  ncclComm_t on its own highest-priority HIP stream, stream-ordered collectives fenced with
  hipEvents (the host never blocks), bootstrapped through the torchrun TCPStore.
* ``TorchComm`` — ``torch.distributed`` (RCCL via ProcessGroupNCCL on GPU, gloo on CPU): the CPU
  test path and the fallback.

Both return work handles whose ``wait()`` orders the caller's current stream after the
collective.  ``get_comm()`` picks native on GPU when the extension is loaded
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


class TorchComm:
    backend = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        if self.world == 1:
            return _Done()
        if op == "avg" and dist.get_backend(self.group) == "gloo":
            w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            w.wait()
            t.div_(self.world)
            return _Done()
        return dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=True)

    def all_reduce_coalesced(self, ts: List[torch.Tensor], op: str = "sum"):
        works = [self.all_reduce(t, op) for t in ts]
        return works[-1] if works else _Done()

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum"):
        if self.world == 1:
            out.copy_(inp)
            return _Done()
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


class NativeComm:
    """Hyperion C++ RCCL communicator bootstrapped over the default TCPStore."""

    backend = "native"
    _counter = 0

    def __init__(self, device: torch.device, group=None, tag: Optional[str] = None):
        C = _native.native()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        NativeComm._counter += 1
        key = f"hyperion_rccl_uid_{tag or NativeComm._counter}"
        store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            store.set(key, C.rccl_unique_id())
        uid = store.get(key)
        self._c = C.RcclComm(bytes(uid), self.rank, self.world, torch.device(device).index or 0)

    @property
    def stream_handle(self) -> int:
        return self._c.stream_handle

    def all_reduce(self, t, op="sum"):
        return self._c.all_reduce(t, op)

    def all_reduce_coalesced(self, ts, op="sum"):
        return self._c.all_reduce_coalesced(list(ts), op)

    def reduce_scatter(self, out, inp, op="sum"):
        return self._c.reduce_scatter(out, inp, op)

    def all_gather(self, out, inp):
        return self._c.all_gather(out, inp)

    def broadcast(self, t, root=0):
        return self._c.broadcast(t, root)

    def all_to_all(self, out, inp):
        return self._c.all_to_all(out, inp)

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
