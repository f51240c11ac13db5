"""Distributed sampler with ``torch.utils.data.DistributedSampler`` semantics.

Reference: ``DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True)`` + ``set_epoch``
in every distributed trainer (``02_development/distributed_utils.py:151,168,225,237,311,339,449,
507``; SURVEY §2.2 "Data sharding").  Same index stream as torch's (``randperm`` seeded with
``seed + epoch``, padding by wrap-around to a multiple of the world size, rank-strided slices), so
runs are comparable sample-for-sample; implemented here so ranks can also be computed without a
process group (used by the synthetic loaders and the CPU tests).
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch
from torch.utils.data import Sampler


class DistributedSampler(Sampler[int]):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            import torch.distributed as dist

            ok = dist.is_available() and dist.is_initialized()
            num_replicas = num_replicas if num_replicas is not None else (dist.get_world_size() if ok else 1)
            rank = rank if rank is not None else (dist.get_rank() if ok else 0)
        if not 0 <= rank < num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if drop_last and n % num_replicas:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def indices(self) -> list:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g).tolist()
        else:
            idx = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad > 0:
                if pad <= len(idx):
                    idx += idx[:pad]
                else:
                    idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        assert len(idx) == self.total_size
        return idx[self.rank : self.total_size : self.num_replicas]

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
