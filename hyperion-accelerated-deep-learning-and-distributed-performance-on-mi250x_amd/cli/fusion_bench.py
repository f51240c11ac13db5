"""CLI twin of the reference's ``compilation_optimization.py --base_dir . --dtype {fp32,bf16} --repeat 10``
(SURVEY C32): eager vs Hyperion-fused vs fused+hipGraph, same models and inputs."""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--base_dir", default=".")
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16", "fp16"])
    ap.add_argument("--repeat", type=int, default=10)
    a = ap.parse_args(argv)
    from hyperion.bench.fusion import run_fusion_benchmark

    run_fusion_benchmark(a.base_dir, a.dtype, a.repeat)
    return 0


if __name__ == "__main__":
    sys.exit(main())
