"""Column-sum (bias gradient) launch forms on the ViT-B/16 / GPT-2 shapes: two launches (partials +
combine) vs one launch with the last-arriver combine at several partial-row caps.  Graph-replayed
(launch gaps included).  python scripts/colsum_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from conv_roofline import gtime  # noqa: E402
from hyperion.ops import _native  # noqa: E402

C = _native.native()
rows = []
for M, N in [(8192, 768), (8192, 3072), (6304, 768), (6304, 3072), (4064, 256), (4064, 2048)]:
    x = torch.randn(M, N, device="cuda").bfloat16()
    r = {"M": M, "N": N}
    for cap in (0, 32, 64, 128):
        C.colsum_set_fused(cap)
        r[f"cap{cap}_us"] = round(gtime(lambda: C.column_sum(x, torch.bfloat16), 20, 5), 2)
    C.colsum_set_fused(64)
    print(json.dumps(r), flush=True)
    rows.append(r)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(rows, open("gpurun_out/colsum_bench.json", "w"), indent=1)
