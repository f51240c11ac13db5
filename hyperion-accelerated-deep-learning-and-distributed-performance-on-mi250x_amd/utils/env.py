"""Runtime / communication environment knobs, documented.

The reference exported ``NCCL_COLLNET_ENABLE=0``, ``RCCL_P2P_ENABLE=1``,
``TORCH_NCCL_ASYNC_ERROR_HANDLING=0`` (watchdog kill OFF), ``TORCH_NCCL_TIMEOUT=7200`` and
``RCCL_TIMEOUT=7200`` in ``run_language_fsdp.sh:8-12``; the two timeout variables are not read by
PyTorch or RCCL, and disabling async error handling makes hangs undetectable.  ``apply_defaults``
sets only knobs that exist, keeps the watchdog ON (failures surface within the process-group
timeout) and leaves anything the user exported untouched.
"""
from __future__ import annotations

import os
from typing import Dict

DEFAULTS: Dict[str, str] = {
    # dmabuf-only IPC on the MI355X hosts (RCCL / CUDA-tensor sharing fails without it)
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    # keep the c10d watchdog: a dead peer turns into an exception instead of a silent hang
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
    # RCCL: fully-connected xGMI fast path; no CollNet on a single node
    "NCCL_COLLNET_ENABLE": "0",
}

DEBUG: Dict[str, str] = {
    "TORCH_DISTRIBUTED_DEBUG": "DETAIL",  # mismatched-collective detection in c10d
    "NCCL_DEBUG": "WARN",
    "AMD_SERIALIZE_KERNEL": "3",          # one kernel at a time: faults point at the right kernel
    "HIP_LAUNCH_BLOCKING": "1",
}


def apply_defaults(debug: bool = False) -> Dict[str, str]:
    applied = {}
    for k, v in {**DEFAULTS, **(DEBUG if debug else {})}.items():
        if k not in os.environ:
            os.environ[k] = v
            applied[k] = v
    return applied
