"""Per-launch time of the stride-1 dgrad with / without the BN-backward epilogue (BNGradLink) per
tile on the ResNet-50 layer1/2 shapes (in-graph, batch 32).  Output: gpurun_out/bnb_tiles.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_variants import gtime  # noqa: E402

C_ = _native.native()
cl = torch.channels_last
rows = []
# (N, K_dy, H, W, C_dx, R, pad, mode): dgrad of a conv K<-C, output [N, C, H, W]
for (N, K, H, W, C, R, p, mode) in [(32, 64, 56, 56, 256, 1, 0, 2), (32, 64, 56, 56, 64, 3, 1, 1),
                                     (32, 256, 56, 56, 64, 1, 0, 1), (32, 128, 28, 28, 512, 1, 0, 2),
                                     (32, 128, 28, 28, 128, 3, 1, 1)]:
    dy = torch.randn(N, K, H, W, device="cuda").bfloat16().contiguous(memory_format=cl)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=cl)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=cl)
    y = torch.relu(x)
    add = torch.randn_like(x) if mode == 2 else None
    bw, bb = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    sums = torch.zeros(8 * 2 * C, device="cuda", dtype=torch.float64)
    r = {"shape": [N, K, H, W, C, R, mode]}
    r["plain_auto"] = gtime(lambda: C_.conv_dgrad(dy, w, p, p, addend=add))
    for bm, bn in [(-1, -1), (64, 64), (128, 64), (128, 128)]:
        key = "bnb_auto" if bm < 0 else f"bnb_{bm}x{bn}"
        r[key] = gtime(lambda: C_.conv_dgrad(dy, w, p, p, bm, bn, -1, add, x, y, bw, bb, mean, inv, mode, sums))
    print(json.dumps(r), flush=True)
    rows.append(r)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(rows, open("gpurun_out/bnb_tiles.json", "w"), indent=1)
