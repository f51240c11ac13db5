"""Distributed runtime: process groups, DDP, FSDP, native RCCL communicator, sampler."""
from .launch import DistEnv, cleanup, dist_env, init_from_env, setup, _local_gpu  # noqa: F401
from .ddp import DDP, DistributedDataParallel  # noqa: F401
