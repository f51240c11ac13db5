"""CLI: hardware exploration (reference ``01_hardware_exploration.ipynb``) on raw HIP kernels.

``python -m hyperion.cli.hardware_bench [--sizes 1024,2048,4096,8192] [--methods proper,reference]
[--out results/benchmarks/hardware]`` → ``precision_results.csv`` + ``bandwidth_results.csv``
(reference schemas + Method/Kernel columns) and a JSON summary of the headline cells.
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--sizes", default="1024,2048,4096,8192")
    ap.add_argument("--bw-sizes", default="10,20,50,100,200,500")
    ap.add_argument("--methods", default="proper,reference")
    ap.add_argument("--kernels", default="hyperion,torch")
    ap.add_argument("--precisions", default="fp32,fp16,bf16")
    ap.add_argument("--bw-ops", default="add,copy,triad")
    ap.add_argument("--out", default="results/benchmarks/hardware")
    a = ap.parse_args(argv)
    from hyperion.bench.hardware import test_gpu_operations, test_memory_bandwidth, test_precision_formats
    from hyperion.utils.device import print_device_info

    print_device_info()
    print("gpu ops:", test_gpu_operations())
    mm = test_precision_formats([int(s) for s in a.sizes.split(",")], a.precisions.split(","), a.kernels.split(","),
                                a.methods.split(","), a.out)
    bw = test_memory_bandwidth([int(s) for s in a.bw_sizes.split(",")], a.bw_ops.split(","), a.kernels.split(","),
                               a.methods.split(","), a.out)
    best = {}
    for r in mm:
        k = f"{r['Method']}/{r['Kernel']}/{r['Precision']}/{r['Size']}"
        best[k] = round(r["TFLOPS"], 2)
    for r in bw:
        k = f"{r['Method']}/{r['Kernel']}/{r['Op']}/{r['Size (M elements)']}M"
        best[k] = round(r["Bandwidth (GB/s)"], 1)
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "hardware_summary.json"), "w") as f:
        json.dump(best, f, indent=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
