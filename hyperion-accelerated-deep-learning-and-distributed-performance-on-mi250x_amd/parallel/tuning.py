"""Collective message sizes chosen from a measured bus-bandwidth curve.

The reference left bucket sizes at PyTorch DDP's defaults (25 MiB buckets, 1 MiB first bucket;
SURVEY §2.6 K3/K4).  On MI355X the xGMI fabric is 7 point-to-point links per GPU, so a ring
all-reduce only reaches its bus bandwidth above some message size that depends on the world size
and on RCCL's channel count — a number to MEASURE, not to copy from NVSwitch systems.

``python -m hyperion.cli.test_rccl --sweep --save-tuning`` (one process per GPU) writes
``configs/busbw_w{world}.json``: the all-reduce / all-gather / reduce-scatter busbw per message
size.  :func:`bucket_mb` then returns the smallest all-reduce message that reaches
``saturation`` (default 90 %) of the best measured busbw — large enough to run at the fabric's
rate, small enough to start overlapping with the backward early.  Without a sweep for the running
world size the caller's default stays (64 MiB DDP buckets: a 288 GB part affords them).
``HYPERION_BUSBW_JSON`` points at another sweep file.
"""
from __future__ import annotations

import json
import os
from typing import Optional

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CONFIG_DIR = os.path.join(_REPO, "configs")


def sweep_path(world: int) -> str:
    return os.environ.get("HYPERION_BUSBW_JSON") or os.path.join(CONFIG_DIR, f"busbw_w{world}.json")


def load_sweep(world: int) -> Optional[dict]:
    p = sweep_path(world)
    if not os.path.isfile(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if int(d.get("world", -1)) != int(world):
        return None
    return d


def saturation_bytes(rows, op: str = "all_reduce", saturation: float = 0.9) -> Optional[int]:
    """Smallest message (bytes) of ``op`` whose busbw is >= ``saturation`` x the best measured."""
    pts = sorted((int(r["bytes"]), float(r["busbw_GBps"])) for r in rows if r.get("op") == op)
    if not pts:
        return None
    best = max(bw for _, bw in pts)
    for nbytes, bw in pts:
        if bw >= saturation * best:
            return nbytes
    return pts[-1][0]


def bucket_mb(world: int, default: float = 64.0, saturation: float = 0.9, lo: float = 4.0, hi: float = 512.0) -> float:
    """DDP bucket size (MiB) for ``world`` ranks: the all-reduce saturation point of the measured
    sweep (clamped to [lo, hi]), or ``default`` when no sweep for this world size exists."""
    d = load_sweep(world)
    if d is None:
        return default
    nb = saturation_bytes(d.get("rows", []), "all_reduce", saturation)
    if nb is None:
        return default
    return float(min(hi, max(lo, nb / 2**20)))
