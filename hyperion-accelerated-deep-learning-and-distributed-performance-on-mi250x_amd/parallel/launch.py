"""Process-group setup / teardown and torchrun environment parsing.

Reference: ``setup``/``cleanup``/``_local_gpu`` in ``02_development/distributed_utils.py:96-125``
(C22) and the env parsing in ``run_distributed.py:73-79``.

Fixes vs the reference:
* the device index comes from ``LOCAL_RANK`` (the reference used ``global_rank % device_count``);
* the timeout is configurable (default 10 min) and the watchdog stays on
  (``TORCH_NCCL_ASYNC_ERROR_HANDLING`` is not forced to 0 as in ``run_language_fsdp.sh:10``);
* backend defaults to ``nccl`` (= RCCL over xGMI) on GPU and ``gloo`` on CPU, so the same code
  is testable without a GPU.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int
    local_world_size: int
    master_addr: str
    master_port: int

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def dist_env() -> DistEnv:
    """Read torchrun's env (defaults: a single process)."""
    return DistEnv(
        rank=int(os.environ.get("RANK", "0")),
        world_size=int(os.environ.get("WORLD_SIZE", "1")),
        local_rank=int(os.environ.get("LOCAL_RANK", "0")),
        local_world_size=int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))),
        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
        master_port=int(os.environ.get("MASTER_PORT", "29500")),
    )


def _local_gpu(rank: int) -> int:
    """Device index for a process (reference name; uses LOCAL_RANK when set)."""
    if "LOCAL_RANK" in os.environ:
        lr = int(os.environ["LOCAL_RANK"])
    else:
        lr = rank
    n = torch.cuda.device_count() if torch.cuda.is_available() else 1
    return lr % max(n, 1)


_TIMEOUT_S = 600.0


def current_timeout_s() -> float:
    """The collective timeout the last ``setup()`` used (the native communicator's deadline)."""
    return _TIMEOUT_S


def default_backend() -> str:
    return "nccl" if torch.cuda.is_available() else "gloo"


def setup(rank: int, world_size: int, backend: Optional[str] = None, timeout_s: float = 600.0) -> torch.device:
    """Create the process group (env:// rendezvous) and bind this process to its GPU."""
    global _TIMEOUT_S
    _TIMEOUT_S = float(timeout_s)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # dmabuf-only IPC on the MI355X hosts; keep legacy IPC off for RCCL (see README)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    backend = backend or default_backend()
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    device = torch.device("cpu")
    if torch.cuda.is_available():
        device = torch.device("cuda", _local_gpu(rank))
        torch.cuda.set_device(device)
    if not dist.is_initialized():
        kw = dict(
            backend=backend,
            init_method="env://",
            rank=rank,
            world_size=world_size,
            timeout=datetime.timedelta(seconds=timeout_s),
        )
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return device


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier()
        finally:
            dist.destroy_process_group()


def init_from_env(backend: Optional[str] = None, timeout_s: float = 600.0) -> DistEnv:
    """torchrun entry: initialize the PG only when WORLD_SIZE > 1; always bind the device."""
    env = dist_env()
    if env.world_size > 1:
        setup(env.rank, env.world_size, backend=backend, timeout_s=timeout_s)
    elif torch.cuda.is_available():
        torch.cuda.set_device(_local_gpu(env.rank))
    return env


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
