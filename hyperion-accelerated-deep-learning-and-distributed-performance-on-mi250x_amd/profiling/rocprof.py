"""rocprofv3 helpers: build the profiling command and summarize kernel traces.

The reference had no profiler integration at all (wall clock only).  These helpers
turn a ``rocprofv3 --kernel-trace --output-format csv`` run into a steady-state per-step kernel
breakdown: the trace is cut into steps at a marker kernel (by default the fused optimizer
``adam_mt_k``, which runs exactly once per training step), warm-up / MIOpen-find dispatches
before the window are dropped, and kernels are grouped into families (conv fwd / dgrad / wgrad,
fused BN, GEMM, optimizer, elementwise …).

CLI: ``python -m hyperion.profiling.rocprof summarize <kernel_trace.csv> [--steps 5] [--marker adam_mt_k]``
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import sys
from collections import defaultdict
from typing import Dict, List, Optional

FAMILIES = [
    ("optimizer", r"adam_mt_k|unscale_mt_k|sumsq_mt_k|clip_mt_k|fused_adam|multi_tensor_apply"),
    ("bn_fused", r"bn_(stats|apply|bwd|eval)"),
    ("layernorm", r"ln_(fwd|bwd)_k|layer_norm|col_sum_k"),
    ("attention", r"attn_|flash|fmha|attention"),
    ("conv_wgrad", r"wrw|bwd_weight|conv.*wgrad|BackwardWeight"),
    ("splitk_reduce", r"splitk_reduce|colsum_"),
    ("conv_dgrad", r"igemm_bwd|bwd_data|conv.*dgrad|BackwardData|conv_fwd_k<[^,]+, \d+, \d+, (true|false), true"),
    ("conv_fwd", r"igemm_fwd|conv_fwd|grouped_conv_fwd|naive_conv.*fwd|ConvFwd|conv2d"),
    ("gemm", r"gemm|Cijk|gemm_mfma|xdl"),
    ("pool", r"pool|gap_(fwd|bwd)"),
    ("embedding", r"embed_"),
    ("softmax_ce", r"softmax|cross_entropy|nll_loss|ce_"),
    ("bn_torch", r"batch_norm|batchnorm|BatchNorm|MIOpenBatchNorm"),
    ("copy_cast", r"copy|Cast|fill"),
    ("elementwise", r"elementwise|Functor|reduce_kernel"),
]


def family(name: str) -> str:
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def load_trace(path: str) -> List[dict]:
    with open(path, newline="") as f:
        rows = list(csv.DictReader(f))
    for r in rows:
        r["start"] = int(r["Start_Timestamp"])
        r["end"] = int(r["End_Timestamp"])
        r["dur"] = r["end"] - r["start"]
    rows.sort(key=lambda r: r["start"])
    return rows


def steady_window(rows: List[dict], marker: str, steps: int) -> List[dict]:
    idx = [i for i, r in enumerate(rows) if re.search(marker, r["Kernel_Name"])]
    if len(idx) < 2:
        return rows
    steps = min(steps, len(idx) - 1)
    lo, hi = idx[-steps - 1], idx[-1]
    return rows[lo + 1 : hi + 1]


def summarize(path: str, steps: int = 5, marker: str = "adam_mt_k", top: int = 25) -> Dict:
    rows = load_trace(path)
    win = steady_window(rows, marker, steps)
    n_steps = max(1, sum(1 for r in win if re.search(marker, r["Kernel_Name"])))
    busy = sum(r["dur"] for r in win)
    span = (win[-1]["end"] - win[0]["start"]) if win else 0
    by_kernel: Dict[str, List[int]] = defaultdict(list)
    by_fam: Dict[str, int] = defaultdict(int)
    for r in win:
        by_kernel[r["Kernel_Name"]].append(r["dur"])
        by_fam[family(r["Kernel_Name"])] += r["dur"]
    kern = sorted(by_kernel.items(), key=lambda kv: -sum(kv[1]))
    return {
        "trace": path,
        "steps": n_steps,
        "kernels_per_step": len(win) / n_steps,
        "gpu_busy_ms_per_step": busy / n_steps / 1e6,
        "span_ms_per_step": span / n_steps / 1e6,
        "families_ms_per_step": {k: round(v / n_steps / 1e6, 4) for k, v in sorted(by_fam.items(), key=lambda kv: -kv[1])},
        "top_kernels": [
            {
                "name": k[:160],
                "family": family(k),
                "calls_per_step": len(v) / n_steps,
                "ms_per_step": round(sum(v) / n_steps / 1e6, 4),
                "avg_us": round(sum(v) / len(v) / 1e3, 2),
            }
            for k, v in kern[:top]
        ],
    }


def format_summary(s: Dict) -> str:
    out = [
        f"trace: {s['trace']}",
        f"steady-state steps: {s['steps']}   kernels/step: {s['kernels_per_step']:.0f}",
        f"GPU busy per step: {s['gpu_busy_ms_per_step']:.3f} ms   span per step: {s['span_ms_per_step']:.3f} ms",
        "",
        "family                 ms/step",
    ]
    for k, v in s["families_ms_per_step"].items():
        out.append(f"  {k:<20} {v:8.3f}")
    out += ["", "  ms/step  calls  avg_us  family        kernel"]
    for k in s["top_kernels"]:
        out.append(
            f"  {k['ms_per_step']:7.3f} {k['calls_per_step']:6.1f} {k['avg_us']:7.1f}  {k['family']:<12}  {k['name'][:100]}"
        )
    return "\n".join(out)


def rocprof_cmd(out_dir: str, program: List[str], pmc: Optional[List[str]] = None, stats: bool = True) -> List[str]:
    """rocprofv3 command line (kernel trace, csv).  PMC runs never add trace domains beyond the
    kernel trace (those combinations are refused on the GPU pool)."""
    cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", out_dir, "-o", "run"]
    if stats:
        cmd.insert(2, "--stats")
    if pmc:
        cmd += ["--pmc"] + list(pmc)
    return cmd + ["--"] + list(program)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("summarize")
    s.add_argument("trace")
    s.add_argument("--steps", type=int, default=5)
    s.add_argument("--marker", default="adam_mt_k")
    s.add_argument("--top", type=int, default=25)
    s.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    summ = summarize(a.trace, a.steps, a.marker, a.top)
    print(format_summary(summ))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(summ, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
