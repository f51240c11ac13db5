"""In-graph per-launch time of the Hyperion conv kernels on every ResNet-50 conv shape (batch 32),
per tile / split configuration: 20 launches captured in one hipGraph, replayed, wall / 20.
The first rows are the automatic plan; then the explicit tiles.  Output: gpurun_out/conv_variants.json

    python scripts/conv_variants.py [fwd,dgrad,wgrad] [--quick]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.bench.conv_shapes import resnet50_convs  # noqa: E402
from hyperion.ops import _native  # noqa: E402

C_ = _native.native()
what = (sys.argv[1] if len(sys.argv) > 1 else "fwd,dgrad,wgrad").split(",")
quick = "--quick" in sys.argv
stages = "--stages" in sys.argv  # automatic plan at LDS ring depths 2, 3, 4


def gtime(fn, n=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


rows = []
for sh in resnet50_convs(32):
    N, C, H, K, R, s, p = sh["N"], sh["C"], sh["H"], sh["K"], sh["R"], sh["stride"], sh["pad"]
    if C % 64:
        continue
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, P, P, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gf = 2.0 * N * P * P * K * C * R * R / 1e9
    r = dict(sh, P=P, gflop=gf)
    tiles = [(0, 0, -1)] + ([] if quick or stages else [(64, 64, 1), (128, 64, 1), (128, 128, 1), (64, 64, -1),
                                                         (128, 64, -1)])
    if stages:
        for nb in (2, 3, 4):
            C_.conv_set_stages(nb, nb)
            r[f"fwd_nb{nb}"] = gtime(lambda: C_.conv_fwd(x, w, s, s, p, p, True))
            if s == 1 and K % 64 == 0:
                r[f"dgrad_nb{nb}"] = gtime(lambda: C_.conv_dgrad(dy, w, p, p))
            r[f"wgrad_nb{nb}"] = gtime(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p))
        C_.conv_set_stages(0, 0)
        rows.append(r)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        continue
    if "fwd" in what:
        for bm, bn, sp in tiles:
            r[f"fwd_{bm}x{bn}_s{sp}"] = gtime(lambda: C_.conv_fwd(x, w, s, s, p, p, True, bm, bn, sp))
    if "dgrad" in what and s == 1 and K % 64 == 0:
        for bm, bn, sp in tiles:
            r[f"dgrad_{bm}x{bn}_s{sp}"] = gtime(lambda: C_.conv_dgrad(dy, w, p, p, bm, bn, sp))
    if "wgrad" in what:
        r["wgrad_auto"] = gtime(lambda: C_.conv_wgrad(dy, x, R, R, s, s, p, p))
    rows.append(r)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(rows, open("gpurun_out/conv_variants.json", "w"), indent=1)
