"""Summarize a rocprofv3 kernel trace of bench.py into per-step families (one adam_mt_k pass marks a step)."""
import collections
import csv
import sys


def fam(n):
    if "conv_fwd_k" in n:
        return "hyp_conv_igemm(fwd+dgrad)"
    if "Cijk" in n:
        return "hipblaslt_gemm"
    if "wrw" in n or "bwd_weight" in n:
        return "miopen_wgrad"
    if "igemm_bwd" in n or "bwd_data" in n:
        return "miopen_dgrad"
    if "igemm_fwd" in n or "grouped_conv_fwd" in n or "naive_conv" in n:
        return "miopen_fwd"
    if "ck::" in n or "kernel_batched_gemm" in n:
        return "ck_gemm"
    if "bn_" in n:
        return "hyp_bn"
    if "adam_mt" in n:
        return "hyp_adam"
    if "at::native" in n:
        return "torch_elementwise"
    return "other"


def main(path, last_steps=5, per_step_markers=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_mt_k" in r["Kernel_Name"]]
    # markers per step = number of adam launches between consecutive optimizer steps
    mps = per_step_markers or 1
    a0, a1 = idx[-(last_steps * mps) - 1], idx[-1]
    win = rows[a0 + 1: a1 + 1]
    t0, t1 = int(rows[a0]["End_Timestamp"]), int(rows[a1]["End_Timestamp"])
    f = collections.defaultdict(float)
    k = collections.defaultdict(lambda: [0, 0.0])
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / last_steps
        f[fam(r["Kernel_Name"])] += d
        key = r["Kernel_Name"][:100]
        k[key][0] += 1
        k[key][1] += d
    print(f"window: {last_steps} steps, span {(t1 - t0) / 1e3 / last_steps:.1f} us/step, busy {sum(f.values()):.1f} us/step,"
          f" {len(win) / last_steps:.0f} kernels/step")
    for name, v in sorted(f.items(), key=lambda x: -x[1]):
        print(f"  {v:8.1f} us  {name}")
    print("top kernels (us/step, calls/step):")
    for name, (n, v) in sorted(k.items(), key=lambda x: -x[1][1])[:25]:
        print(f"  {v:8.1f} {n / last_steps:5.1f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5, int(sys.argv[3]) if len(sys.argv) > 3 else None)
