"""Run ids, reference-schema metric CSVs, and JSON run manifests.

Reference schemas: ``{model}_{world}gpus_{YYYYmmdd_HHMMSS}`` run ids
(``distributed_utils.py:140,215,301,438``) and per-epoch CSVs:

* LM DDP / FSDP: ``epoch,loss,duration,gpus`` (:147, :306)
* CIFAR DDP: ``epoch,loss,accuracy,duration,gpus`` (:222)
* Llama: ``epoch,loss,duration_s,gpus,mode`` (:443)

The same files are written here (rank 0 only) so ``create_scaling_report`` and the reference's
plots read them unchanged; a sidecar ``{run_id}_run.json`` adds what the reference never logged
(samples/s, tokens/s, step ms, peak memory, device/arch/RCCL versions, git SHA).
"""
from __future__ import annotations

import csv
import json
import os
import subprocess
import time
from typing import Dict, List, Optional

SCHEMAS: Dict[str, List[str]] = {
    "language_ddp": ["epoch", "loss", "duration", "gpus"],
    "language_fsdp": ["epoch", "loss", "duration", "gpus"],
    "gpt2_fsdp": ["epoch", "loss", "duration", "gpus"],
    "cifar": ["epoch", "loss", "accuracy", "duration", "gpus"],
    "llama": ["epoch", "loss", "duration_s", "gpus", "mode"],
}


def make_run_id(model: str, world: int, when: Optional[float] = None) -> str:
    return f"{model}_{world}gpus_{time.strftime('%Y%m%d_%H%M%S', time.localtime(when))}"


class MetricsCSV:
    def __init__(self, path: str, columns: List[str], enabled: bool = True, append: bool = False):
        """``append``: continue an existing file (a resumed run keeps its run_id and CSV)."""
        self.path = path
        self.columns = columns
        self.enabled = enabled
        if enabled and not (append and os.path.exists(path)):
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path, "w", newline="") as f:
                csv.writer(f).writerow(columns)

    def append(self, **row) -> None:
        if not self.enabled:
            return
        with open(self.path, "a", newline="") as f:
            csv.writer(f).writerow([row[c] for c in self.columns])


def git_sha(repo: Optional[str] = None) -> Optional[str]:
    try:
        return subprocess.run(["git", "rev-parse", "HEAD"], cwd=repo or os.path.dirname(__file__), capture_output=True,
                              text=True, timeout=5).stdout.strip() or None
    except Exception:
        return None


def write_manifest(path: str, payload: Dict) -> None:
    from ..utils.device import device_info

    doc = {"device": device_info(), "git_sha": git_sha(), "time": time.time()}
    doc.update(payload)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(doc, f, indent=2, default=str)
