"""Device-side input pipeline: pinned host batches copied on a side HIP stream, one batch ahead.

The reference's loaders (``DataLoader(bs, num_workers=2)`` + ``ids.to(dev)`` from pageable memory
inside the hot loop, ``distributed_utils.py:152,171``) serialise the H2D copy with compute.
``DevicePrefetcher`` pins each batch, issues its copy on a dedicated copy stream while the
previous step computes, and hands the compute stream an event-ordered device batch
(``record_stream`` keeps the caching allocator honest).  On CPU it is a pass-through.
"""
from __future__ import annotations

from typing import Any, Iterable, Iterator, Optional

import torch


def _to(obj: Any, device: torch.device, non_blocking: bool):
    if isinstance(obj, torch.Tensor):
        if device.type == "cuda" and not obj.is_cuda and not obj.is_pinned():
            obj = obj.pin_memory()
        return obj.to(device, non_blocking=non_blocking)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to(o, device, non_blocking) for o in obj)
    if isinstance(obj, dict):
        return {k: _to(v, device, non_blocking) for k, v in obj.items()}
    return obj


def _record(obj: Any, stream) -> None:
    if isinstance(obj, torch.Tensor) and obj.is_cuda:
        obj.record_stream(stream)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _record(o, stream)
    elif isinstance(obj, dict):
        for o in obj.values():
            _record(o, stream)


class DevicePrefetcher:
    def __init__(self, loader: Iterable, device: torch.device):
        self.loader = loader
        self.device = torch.device(device)
        self.stream: Optional[torch.cuda.Stream] = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def __len__(self) -> int:
        return len(self.loader)  # type: ignore[arg-type]

    def __iter__(self) -> Iterator:
        if self.stream is None:
            for b in self.loader:
                yield _to(b, self.device, False)
            return
        it = iter(self.loader)
        nxt = self._preload(it)
        while nxt is not None:
            cur_stream = torch.cuda.current_stream(self.device)
            cur_stream.wait_stream(self.stream)
            batch = nxt
            _record(batch, cur_stream)
            nxt = self._preload(it)
            yield batch

    def _preload(self, it):
        try:
            b = next(it)
        except StopIteration:
            return None
        with torch.cuda.stream(self.stream):
            return _to(b, self.device, True)
