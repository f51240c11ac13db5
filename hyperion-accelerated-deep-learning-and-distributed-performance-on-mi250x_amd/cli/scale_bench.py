"""Headline scaling run: ``bench.py`` (ResNet-50 bf16 training, BASELINE.json) at several GPU
counts, one fresh child per count, then ``scaling_resnet50.csv`` (gpus, samples_per_s,
ms_per_step, speedup, efficiency, replicas_in_sync) — the reference's scaling experiment
(``02_development/distributed_utils.py:563-773, 780-831``) for the headline metric.

    python -m hyperion.cli.scale_bench --gpus 1,2,4,8 [--out results/scaling] [-- <bench.py args>]
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--out", default="results/scaling")
    ap.add_argument("--timeout", type=float, default=1800.0, help="seconds per GPU count")
    a = ap.parse_args(argv)
    from hyperion.bench.scaling import run_bench_scaling

    res = run_bench_scaling([int(g) for g in a.gpus.split(",")], a.out, extra, a.timeout)
    return 0 if res else 1


if __name__ == "__main__":
    sys.exit(main())
