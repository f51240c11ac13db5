"""Multi-tensor launch tables for the gfx950 multi-tensor kernels (``csrc/kernels/adam.hip``).

A table is built once per set of tensor pointers and reused while the pointers stay the same.
Each row of the block table is (tensor id, chunk id); one 256-thread block processes ``chunk``
elements.

hipGraph capture: a table is never ALLOCATED during capture (see ``MultiTensorTable``), but one
built during warm-up can be RE-POINTED there — same tensor count and sizes, new addresses (the
captured step's gradients: ``TrainStep`` lets autograd steal the fresh weight gradients instead of
adding them into kept ``.grad`` buffers, which cost one add kernel per parameter per step).  The
captured kernel reads the table's device buffer at replay time, so the new pointers are written
into that (pre-capture) buffer right after capture ends: ``flush_pending()``.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch

CHUNK = 8192  # elements per block (multiple of 4 for the float4 body)



_PENDING: List[Tuple[torch.Tensor, torch.Tensor]] = []  # (device pointer table, host pointers)


def flush_pending() -> int:
    """Write the pointer updates recorded during a hipGraph capture (call after the capture ends,
    before the first replay); returns how many tables were updated."""
    n = len(_PENDING)
    for dev_t, host_t in _PENDING:
        dev_t.copy_(host_t)
    _PENDING.clear()
    return n


class MultiTensorTable:
    def __init__(self, groups: Sequence[Sequence[torch.Tensor]], chunk: int = CHUNK):
        """``groups``: K lists of T tensors each (e.g. [params, grads, exp_avg, exp_avg_sq])."""
        assert groups and all(len(g) == len(groups[0]) for g in groups)
        self.layout = self.layout_of(groups)
        self.T = len(groups[0])
        self.chunk = chunk
        dev = groups[0][0].device
        self.key = self.key_of(groups)
        ptrs = [t.data_ptr() for g in groups for t in g]
        for p in ptrs:
            if p % 16:
                raise ValueError("multi-tensor kernels need 16-byte aligned tensors")
        sizes = [t.numel() for t in groups[0]]
        blocks: List[int] = []
        for i, n in enumerate(sizes):
            for c in range((n + chunk - 1) // chunk):
                blocks += [i, c]
        self.nblocks = len(blocks) // 2
        if not blocks:
            blocks = [0, 0]
        host = [
            torch.tensor(ptrs, dtype=torch.int64),
            torch.tensor(sizes, dtype=torch.int64),
            torch.tensor(blocks, dtype=torch.int32).view(-1, 2),
        ]
        if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            # A table allocated inside a hipGraph capture lives in the graph's private pool, and
            # that pool recycles blocks freed EARLIER in the capture: on every replay the kernels
            # that used the block before would overwrite the pointer table (illegal address).
            # Tables must therefore exist before capture, over tensors whose addresses the
            # captured step keeps (TrainStep keeps .grad allocated and zeroes it in place).
            raise RuntimeError(
                "hyperion: multi-tensor table built during hipGraph capture; tensor addresses changed "
                "since warm-up (keep .grad allocated: zero_grad(set_to_none=False) inside the captured step)"
            )
        dev_t = [_h2d(h, dev) for h in host]
        self.ptrs, self.sizes, self.blocks = dev_t
        if self.nblocks == 0:
            self.blocks = self.blocks[:0]

    @staticmethod
    def key_of(groups: Sequence[Sequence[torch.Tensor]]) -> Tuple[int, ...]:
        return tuple(t.data_ptr() for g in groups for t in g)

    @staticmethod
    def layout_of(groups: Sequence[Sequence[torch.Tensor]]) -> Tuple:
        return (len(groups),) + tuple(t.numel() for t in groups[0])

    def repoint(self, groups: Sequence[Sequence[torch.Tensor]]) -> None:
        """Same tensor count and sizes, new addresses: rewrite the pointer table in place (the
        block table depends on sizes only).  Deferred to ``flush_pending`` under capture."""
        ptrs = [t.data_ptr() for g in groups for t in g]
        if any(p % 16 for p in ptrs):
            raise ValueError("multi-tensor kernels need 16-byte aligned tensors")
        host = torch.tensor(ptrs, dtype=torch.int64)
        if self.ptrs.is_cuda and torch.cuda.is_current_stream_capturing():
            _PENDING.append((self.ptrs, host))
        elif self.ptrs.is_cuda:
            # stream-ordered, no host sync: with set_to_none gradients every eager step re-points
            # the table, and a blocking pageable copy stalled the host until the backward drained
            # (the next step's launches then started from an idle GPU: ViT-B/16 fp32 "optimizer
            # time" 6.6 ms vs torch's 1.6 ms, profiles/r04/models)
            self.ptrs.copy_(host.pin_memory(), non_blocking=True)
        else:
            self.ptrs.copy_(host)
        self.key = self.key_of(groups)


def _h2d(h: torch.Tensor, dev: torch.device) -> torch.Tensor:
    if dev.type != "cuda":
        return h.to(dev)
    return h.pin_memory().to(dev, non_blocking=True)  # pinned block reused once the copy's event passed


def _capturing(dev) -> bool:
    return dev is not None and dev.type == "cuda" and torch.cuda.is_current_stream_capturing()


class TableCache:
    """Keeps the most recent table per role; rebuilds (or re-points) when pointers change.

    A table that a hipGraph capture used is PINNED: the captured kernel reads its device pointer
    buffer at every replay, so it is never re-pointed or dropped afterwards (the cache, owned by
    the optimizer / model whose graph it is, keeps it alive).  An eager call with other pointers
    after that gets a table of its own, so it can never redirect the graph's kernel to other
    (possibly freed) tensors.
    """

    def __init__(self):
        self._tables: Dict[str, MultiTensorTable] = {}
        self._pinned: Dict[str, List[MultiTensorTable]] = {}

    def get(self, role: str, groups: Sequence[Sequence[torch.Tensor]]) -> MultiTensorTable:
        key = MultiTensorTable.key_of(groups)
        capturing = _capturing(groups[0][0].device if groups and groups[0] else None)
        t = self._tables.get(role)
        if t is None or t.key != key:
            hit = next((p for p in self._pinned.get(role, ()) if p.key == key), None)
            if hit is not None:
                t = hit
            elif t is not None and not getattr(t, "pinned", False) and t.layout == MultiTensorTable.layout_of(groups):
                t.repoint(groups)
            else:
                t = MultiTensorTable(groups)  # raises under capture (no allocation in the graph pool)
            self._tables[role] = t
        if capturing and not getattr(t, "pinned", False):
            t.pinned = True
            self._pinned.setdefault(role, []).append(t)
        return t

    def pinned(self) -> List[MultiTensorTable]:
        return [t for ts in self._pinned.values() for t in ts]
