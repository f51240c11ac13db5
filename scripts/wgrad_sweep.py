"""Weight-gradient tile / split sweep over the distinct ResNet-50 (batch 32) conv shapes: in-graph
per-launch time (kernel + split-K reduce) for every (BM, BN) tile and pixel-split depth, next to the
automatic plan.  Output: gpurun_out/wgrad_sweep.json

    python scripts/wgrad_sweep.py [--batch 32]
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.bench.conv_shapes import resnet50_convs  # noqa: E402
from hyperion.ops import _native  # noqa: E402
from scripts.gemm_shapes import gtime  # noqa: E402

C_ = _native.native()
batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 32

rows, seen = [], set()
from collections import Counter  # noqa: E402


def _counts():
    from hyperion.models.resnet import resnet50
    m, c, h = resnet50(), Counter(), 56
    for layer in (m.layer1, m.layer2, m.layer3, m.layer4):
        for blk in layer:
            for conv, hin in ((blk.conv1, h), (blk.conv2, h), (blk.conv3, None)):
                hin = hin if hin is not None else h2
                c[(conv.in_channels, hin, conv.out_channels, conv.kernel_size[0], conv.stride[0])] += 1
                if conv is blk.conv2:
                    h2 = (hin + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
            if blk.downsample is not None:
                d = blk.downsample[0]
                c[(d.in_channels, h, d.out_channels, d.kernel_size[0], d.stride[0])] += 1
            h = h2
    return c


count = _counts()
for sh in resnet50_convs(batch):
    N, C, H, K, R, s, p = sh["N"], sh["C"], sh["H"], sh["K"], sh["R"], sh["stride"], sh["pad"]
    key = (C, H, K, R, s)
    if C % 64 or key in seen:
        continue
    seen.add(key)
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    steps = (N * P * P + 63) // 64
    r = dict(C=C, H=H, K=K, R=R, stride=s, count=count[key], M=N * P * P, gflop=2.0 * N * P * P * K * C * R * R / 1e9)
    r["auto"] = gtime(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p))
    best = ("auto", r["auto"])
    for bm, bn in ((64, 64), (128, 64), (64, 128), (128, 128)):
        if C % bn or (bm == 128 and K < 128):
            continue
        for per in (6, 8, 12, 16, 24, 32, 48):
            sp = math.ceil(steps / per)
            if sp > 256:
                continue
            t = gtime(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p, bm, bn, sp))
            name = f"{bm}x{bn}_per{per}_sp{sp}"
            r[name] = t
            if t < best[1]:
                best = (name, t)
    r["best"] = best[0]
    r["best_us"] = best[1]
    r["best_tflops"] = r["gflop"] / best[1] * 1e3
    rows.append(r)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()
                      if not k[0].isdigit()}), flush=True)

tot_auto = sum(r["auto"] * r["count"] for r in rows)
tot_best = sum(r["best_us"] * r["count"] for r in rows)
print(json.dumps({"sum_auto_us": round(tot_auto, 1), "sum_best_us": round(tot_best, 1)}))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(rows, open("gpurun_out/wgrad_sweep.json", "w"), indent=1)
