"""Distributed runtime: process groups, DDP, FSDP, native RCCL communicator, sampler."""
from .ddp import DDP, DistributedDataParallel  # noqa: F401
from .fsdp import (  # noqa: F401
    FSDP,
    FullyShardedDataParallel,
    MixedPrecision,
    size_based_auto_wrap_policy,
    transformer_auto_wrap_policy,
)
from .launch import DistEnv, _local_gpu, cleanup, dist_env, init_from_env, setup  # noqa: F401
