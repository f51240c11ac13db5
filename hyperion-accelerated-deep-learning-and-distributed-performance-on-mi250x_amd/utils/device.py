"""Device / architecture probe (reference C1: ``01_hardware_exploration.ipynb:151-168``,
``core_framework.ipynb:22-36``).

Differences from the reference:
* the local device comes from ``LOCAL_RANK`` (the reference used ``global_rank % device_count``,
  ``distributed_utils.py:96-98``, which breaks on multi-node);
* the probe reports the gfx arch, CU count and HBM size so a run manifest can prove it ran on
  gfx950.
"""
from __future__ import annotations

import os
import platform
import sys
from typing import Any, Dict

import torch


def on_gpu() -> bool:
    return torch.cuda.is_available()


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def get_device(rank: int | None = None) -> torch.device:
    """Device for this process: ``cuda:LOCAL_RANK`` on a GPU box, CPU otherwise."""
    if not torch.cuda.is_available():
        return torch.device("cpu")
    idx = local_rank() if rank is None else rank
    idx = idx % max(torch.cuda.device_count(), 1)
    return torch.device("cuda", idx)


def gcn_arch(idx: int = 0) -> str:
    if not torch.cuda.is_available():
        return "cpu"
    props = torch.cuda.get_device_properties(idx)
    return getattr(props, "gcnArchName", "unknown").split(":")[0]


def is_gfx950(idx: int = 0) -> bool:
    return gcn_arch(idx) == "gfx950"


def get_gpu_memory(idx: int = 0) -> Dict[str, float]:
    """Allocated / reserved / peak memory in MB (reference ``get_gpu_memory`` :161-164)."""
    if not torch.cuda.is_available():
        return {"allocated_mb": 0.0, "reserved_mb": 0.0, "peak_mb": 0.0}
    return {
        "allocated_mb": torch.cuda.memory_allocated(idx) / 2**20,
        "reserved_mb": torch.cuda.memory_reserved(idx) / 2**20,
        "peak_mb": torch.cuda.max_memory_allocated(idx) / 2**20,
    }


def device_info() -> Dict[str, Any]:
    """Versions + per-GPU properties (name, arch, CUs, HBM)."""
    info: Dict[str, Any] = {
        "python": sys.version.split()[0],
        "platform": platform.platform(),
        "torch": torch.__version__,
        "hip": getattr(torch.version, "hip", None),
        "cuda_available": torch.cuda.is_available(),
        "gpus": [],
    }
    if torch.cuda.is_available():
        try:
            info["rccl"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:  # pragma: no cover - depends on build
            info["rccl"] = None
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            info["gpus"].append(
                {
                    "index": i,
                    "name": p.name,
                    "arch": getattr(p, "gcnArchName", "unknown"),
                    "compute_units": p.multi_processor_count,
                    "hbm_gb": round(p.total_memory / 1e9, 1),
                }
            )
    return info


def print_device_info() -> None:
    info = device_info()
    print(f"PyTorch {info['torch']}  HIP {info['hip']}  Python {info['python']}")
    print(f"Number of GPUs: {len(info['gpus'])}")
    for g in info["gpus"]:
        print(f"GPU {g['index']}: {g['name']} ({g['arch']}, {g['compute_units']} CUs, {g['hbm_gb']} GB)")
