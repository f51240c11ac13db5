"""Distributed consistency checks (the reference had no desync detection although
README.md:256 names "silent desync" as a failure mode).

* ``replica_checksums`` / ``assert_replicas_in_sync`` — per-parameter fp64 checksums all-gathered
  and compared across ranks (DDP replicas must be bit-identical after every step);
* ``assert_same_collective_sequence`` — all-gathers a hash of a caller-supplied tag so ranks that
  diverge in control flow (and would issue mismatched collectives, like the reference's rank-0-only
  FSDP state-dict gather, K13) fail fast with a readable error instead of hanging.
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def replica_checksums(params: Iterable[torch.Tensor]) -> torch.Tensor:
    """[n_params, 2] fp64 (Σx, Σx²) per tensor: identical replicas give identical rows (the sums run
    in one fixed order on one device type), and a differing element moves at least one of them."""
    rows = []
    for p in params:
        d = p.detach().double()
        rows.append(torch.stack([d.sum(), (d * d).sum()]))
    return torch.stack(rows) if rows else torch.zeros(0, 2, dtype=torch.float64)


def assert_replicas_in_sync(model: nn.Module, group=None, atol: float = 0.0) -> int:
    """Raise if any parameter differs between ranks; returns the number of tensors compared."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return 0
    inner = getattr(model, "module", model)
    cs = replica_checksums(inner.parameters())
    dev = next(inner.parameters()).device
    cs = cs.to(dev)
    world = dist.get_world_size(group)
    out = [torch.empty_like(cs) for _ in range(world)]
    dist.all_gather(out, cs, group=group)
    names = [n for n, _ in inner.named_parameters()]
    for r in range(1, world):
        diff = (out[r] - out[0]).abs().amax(dim=1) if cs.dim() == 2 else (out[r] - out[0]).abs()
        bad = (diff > atol).nonzero().flatten().tolist()
        if bad:
            raise RuntimeError(f"replica desync: rank {r} differs from rank 0 in {[names[i] for i in bad[:5]]}"
                               f"{' ...' if len(bad) > 5 else ''}")
    return len(names)


def assert_same_collective_sequence(tag: str, group=None, device: Optional[torch.device] = None) -> None:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    h = int(hashlib.sha1(tag.encode()).hexdigest()[:12], 16)
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                     and dist.get_backend(group) == "nccl" else torch.device("cpu"))
    t = torch.tensor([h], dtype=torch.int64, device=dev)
    out: List[torch.Tensor] = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    vals = [int(o.item()) for o in out]
    if len(set(vals)) != 1:
        raise RuntimeError(f"collective sequence mismatch at '{tag}': per-rank tags {vals}")
