"""Kernel-level split of the weight-gradient cost (conv_wgrad_k vs its split-K reduce) on a few
ResNet-50 (batch 32) shapes, per tile / split / LDS ring depth.  Run under rocprofv3:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wprobe -o run -- python3 scripts/wgrad_probe.py
    python3 scripts/wgrad_probe.py --parse gpurun_out/wprobe/run_kernel_trace.csv

The run writes the launch plan (label, launches) to gpurun_out/wgrad_probe_plan.json; --parse walks
the trace in order and prints the median duration of each config's wgrad and reduce kernels.
"""
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REPS = 6
SHAPES = [  # C, H, K, R, stride
    (64, 56, 256, 1, 1), (64, 56, 64, 3, 1), (256, 56, 64, 1, 1), (128, 28, 128, 3, 1), (512, 28, 128, 1, 1),
    (1024, 14, 256, 1, 1), (256, 14, 1024, 1, 1), (256, 14, 256, 3, 1), (512, 7, 512, 3, 1), (2048, 7, 512, 1, 1),
]
CONFIGS = [  # bm, bn, splits (-1 auto / per-steps target when negative < -1), nb (| 8: per-tile stage
    # (unused), | 16: dense shapes on the general kernel, | 32: 128-pixel stages in the dense kernel)
    (64, 64, -1, 2), (64, 64, -1, 2 | 32), (64, 64, -1, 3 | 32), (64, 64, -32, 3 | 32), (128, 64, -16, 2 | 32),
    (128, 64, -16, 3 | 32), (128, 64, -32, 3 | 32), (128, 128, -16, 2 | 32), (128, 128, -32, 2 | 32),
    (64, 128, -16, 3 | 32),
]
DENSE_ONLY = True


def run():
    import torch
    from hyperion.ops import _native
    C_ = _native.native()
    plan = []
    for (C, H, K, R, s) in SHAPES:
        if DENSE_ONLY and (R != 1 or s != 1):
            continue
        p = R // 2
        P = (H + 2 * p - R) // s + 1
        N = 32
        x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        steps = (N * P * P + 63) // 64
        for bm, bn, sp, nb in CONFIGS:
            if C % bn or K < bm:
                continue
            if sp < -1:
                sp = (steps + (-sp) - 1) // (-sp)
            C_.conv_set_stages(0, nb)
            for _ in range(REPS):
                C_.conv_wgrad(dy, x, R, R, s, s, p, p, bm if sp != -1 or bm != 64 else -1, bn, sp)
            torch.cuda.synchronize()
            plan.append(dict(shape=[C, H, K, R, s], bm=bm, bn=bn, splits=sp, nb=nb, reps=REPS))
    C_.conv_set_stages(0, 0)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(plan, open("gpurun_out/wgrad_probe_plan.json", "w"))


def parse(path):
    plan = json.load(open("gpurun_out/wgrad_probe_plan.json"))
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "conv_wgrad_" in r["Kernel_Name"] or ("splitk_reduce_k" in r["Kernel_Name"] or "splitk_reduce4_k" in r["Kernel_Name"])]
    i, out = 0, []
    for p in plan:
        wk, rd = [], []
        for _ in range(p["reps"]):
            w = rows[i]
            assert "conv_wgrad_" in w["Kernel_Name"], w["Kernel_Name"]
            wk.append((int(w["End_Timestamp"]) - int(w["Start_Timestamp"])) / 1e3)
            i += 1
            if i < len(rows) and ("splitk_reduce_k" in rows[i]["Kernel_Name"] or "splitk_reduce4_k" in rows[i]["Kernel_Name"]):
                rd.append((int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3)
                i += 1
        r = dict(p, wgrad_us=round(statistics.median(wk[1:]), 2),
                 reduce_us=round(statistics.median(rd[1:]), 2) if len(rd) > 1 else 0.0)
        out.append(r)
        print(json.dumps(r))
    json.dump(out, open(os.path.join(os.path.dirname(path), "wgrad_probe.json"), "w"), indent=1)


def one(spec):
    """--one C,H,K,R,s,bm,bn,splits,nb: 20 launches of one config (PMC passes) + hipBLASLt dYᵀ·X
    for 1x1 shapes (the vendor GEMM on the same operands, for scale)"""
    import torch
    from hyperion.ops import _native
    C_ = _native.native()
    C, H, K, R, s, bm, bn, sp, nb = (int(v) for v in spec.split(","))
    p = R // 2
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(32, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(32, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    C_.conv_set_stages(0, nb)
    for _ in range(20):
        C_.conv_wgrad(dy, x, R, R, s, s, p, p, bm, bn, sp)
    if R == 1 and s == 1:
        a = dy.permute(0, 2, 3, 1).reshape(-1, K)
        b = x.permute(0, 2, 3, 1).reshape(-1, C)
        for _ in range(20):
            torch.mm(a.t(), b)
    torch.cuda.synchronize()


if __name__ == "__main__":
    if "--one" in sys.argv:
        one(sys.argv[sys.argv.index("--one") + 1])
    elif "--parse" in sys.argv:
        parse(sys.argv[sys.argv.index("--parse") + 1])
    else:
        run()
