"""amd-smi / rocm-smi sampling during a run (SURVEY §5.5 MI355X plan: power and clock sampling).

The reference logged only wall clock and ``torch.cuda`` memory counters.  ``SmiSampler`` polls
``amd-smi metric --json`` (falling back to ``rocm-smi --showpower --showclocks --json``) on a
background thread and records per-GPU power (W), GFX clock (MHz), junction temperature (°C) and
VRAM used (MiB); ``summary()`` reduces the samples to mean / max per metric.  Missing tools or
unparseable output degrade to an empty record — never an exception in a training loop.

    with SmiSampler(interval_s=0.5) as smi:
        run_benchmark()
    print(smi.summary())
"""
from __future__ import annotations

import json
import shutil
import subprocess
import threading
import time
from typing import Dict, List, Optional

_KEYS = {
    "power_w": ("socket_power", "average_socket_power", "current_socket_power", "power"),
    "gfx_clock_mhz": ("gfx_0", "gfxclk", "current_gfxclk", "sclk"),
    "temp_c": ("hotspot", "junction", "edge"),
    "vram_used_mib": ("used_vram", "vram_used"),
}


def _num(v) -> Optional[float]:
    if isinstance(v, dict):
        for k in ("value", "clk", "current"):
            if k in v:
                return _num(v[k])
        return None
    try:
        return float(str(v).split()[0])
    except (TypeError, ValueError, IndexError):
        return None


def _find(d, names) -> Optional[float]:
    """Depth-first search of a nested amd-smi JSON record for the first key among ``names``."""
    if isinstance(d, dict):
        for k, v in d.items():
            if k.lower() in names:
                n = _num(v)
                if n is not None:
                    return n
        for v in d.values():
            n = _find(v, names)
            if n is not None:
                return n
    elif isinstance(d, list):
        for v in d:
            n = _find(v, names)
            if n is not None:
                return n
    return None


def parse_amd_smi(text: str) -> List[Dict[str, float]]:
    """One dict of metrics per GPU from ``amd-smi metric --json`` output."""
    try:
        data = json.loads(text)
    except json.JSONDecodeError:
        return []
    gpus = data if isinstance(data, list) else data.get("gpu_data", [data]) if isinstance(data, dict) else []
    out = []
    for g in gpus:
        rec = {}
        for key, names in _KEYS.items():
            v = _find(g, tuple(n.lower() for n in names))
            if v is not None:
                rec[key] = v
        out.append(rec)
    return out


def sample_once(timeout_s: float = 10.0) -> List[Dict[str, float]]:
    if shutil.which("amd-smi"):
        try:
            r = subprocess.run(["amd-smi", "metric", "--json"], capture_output=True, text=True, timeout=timeout_s)
            recs = parse_amd_smi(r.stdout)
            if recs:
                return recs
        except (OSError, subprocess.TimeoutExpired):
            pass
    if shutil.which("rocm-smi"):
        try:
            r = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--showtemp", "--json"],
                               capture_output=True, text=True, timeout=timeout_s)
            data = json.loads(r.stdout)
            out = []
            for _, card in sorted(data.items()):
                rec = {}
                for k, v in card.items():
                    lk = k.lower()
                    n = _num(str(v).strip("()Mhz"))
                    if n is None:
                        continue
                    if "power" in lk:
                        rec["power_w"] = n
                    elif "sclk" in lk:
                        rec["gfx_clock_mhz"] = n
                    elif "junction" in lk or "hotspot" in lk:
                        rec["temp_c"] = n
                out.append(rec)
            return out
        except (OSError, subprocess.TimeoutExpired, json.JSONDecodeError, AttributeError):
            pass
    return []


class SmiSampler:
    def __init__(self, interval_s: float = 1.0):
        self.interval_s = interval_s
        self.samples: List[List[Dict[str, float]]] = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def _loop(self) -> None:
        while not self._stop.is_set():
            t0 = time.time()
            s = sample_once()
            if s:
                self.samples.append(s)
            self._stop.wait(max(0.0, self.interval_s - (time.time() - t0)))

    def __enter__(self) -> "SmiSampler":
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()
        return self

    def __exit__(self, *exc) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=15)

    def summary(self) -> Dict[str, Dict[str, float]]:
        """{"gpu0.power_w": {"mean": .., "max": ..}, ...} over all samples."""
        acc: Dict[str, List[float]] = {}
        for snap in self.samples:
            for i, rec in enumerate(snap):
                for k, v in rec.items():
                    acc.setdefault(f"gpu{i}.{k}", []).append(v)
        return {k: {"mean": sum(v) / len(v), "max": max(v), "n": len(v)} for k, v in acc.items()}
