"""Fault injection for failure-detection tests (SURVEY §5.3 MI355X plan).

``HYPERION_FAULT=rank:step:kind`` makes the given rank misbehave at the given training step:
``exit`` (process dies with status 17), ``raise`` (Python exception), ``hang`` (sleeps far past
the process-group timeout), ``nan`` (returns True so the caller poisons its loss).  Trainers call
:func:`maybe_inject` once per step; tests assert that the surviving ranks fail within the
configured timeout instead of hanging (the reference disabled the watchdog:
``TORCH_NCCL_ASYNC_ERROR_HANDLING=0``, ``run_language_fsdp.sh:10``).

``stall`` is the GPU-side fault of the native communicator (``parallel/comm.py``): the given rank's
comm stream sleeps ``HYPERION_FAULT_STALL_S`` seconds (default 30) on the device ahead of its
``step``-th collective (here ``step`` counts that communicator's collectives), so peers — or, at
world 1, the rank itself — miss the collective deadline and the watchdog must fail it cleanly.

``HYPERION_FAULT_MARKER=path`` makes the fault one-shot across restarts: it fires only while the
marker file does not exist and creates it when it fires (restart + auto-resume tests: the resumed
run replays the same step numbers and must not fail again).
"""
from __future__ import annotations

import os
import sys
import time
from typing import Optional, Tuple


def parse(spec: Optional[str] = None) -> Optional[Tuple[int, int, str]]:
    spec = spec if spec is not None else os.environ.get("HYPERION_FAULT", "")
    if not spec:
        return None
    r, s, k = spec.split(":")
    if k not in ("exit", "raise", "hang", "nan", "stall"):
        raise ValueError(f"unknown fault kind {k!r}")
    return int(r), int(s), k


class InjectedFault(RuntimeError):
    pass


def comm_stall_s(rank: int, seq: int, spec: Optional[str] = None) -> float:
    """Seconds of device stall to inject before this rank's seq-th native collective (0 = none)."""
    f = parse(spec)
    if f is None or f[2] != "stall" or f[0] != rank or f[1] != seq:
        return 0.0
    return float(os.environ.get("HYPERION_FAULT_STALL_S", "30"))


def maybe_inject(rank: int, step: int, spec: Optional[str] = None) -> bool:
    f = parse(spec)
    if f is None or f[0] != rank or f[1] != step or f[2] == "stall":
        return False
    marker = os.environ.get("HYPERION_FAULT_MARKER")
    if marker:
        if os.path.exists(marker):
            return False
        with open(marker, "w") as fh:
            fh.write(f"{rank}:{step}\n")
    kind = f[2]
    if kind == "exit":
        sys.stderr.write(f"[hyperion] injected fault: rank {rank} exits at step {step}\n")
        sys.stderr.flush()
        os._exit(17)
    if kind == "raise":
        raise InjectedFault(f"injected fault at rank {rank} step {step}")
    if kind == "hang":
        time.sleep(float(os.environ.get("HYPERION_FAULT_HANG_S", "3600")))
        return False
    return True  # nan
