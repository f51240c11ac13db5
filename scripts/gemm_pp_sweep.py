"""Native tiles (classic gemm_tile_k and ping-pong gemm_pp_k) vs the vendor GEMM per shape and
layout, warm device time (median of 10 event-timed calls on randn operands):

    python scripts/gemm_pp_sweep.py [--big] > gpurun_out/.../sweep.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from hyperion.ops import _native  # noqa: E402

C = _native.native()


def t_us(fn, reps=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    torch.cuda._sleep(1_000_000)
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return sorted(s.elapsed_time(e) for s, e in ev)[reps // 2] * 1e3


# (layout, M, N, K): forward NT x W^T, data-gradient NN dy W, weight-gradient TN dy^T x
SHAPES = [
    ("nt", 6304, 2304, 768), ("nt", 6304, 768, 768), ("nt", 6304, 3072, 768), ("nt", 6304, 768, 3072),
    ("nn", 6304, 768, 2304), ("nn", 6304, 768, 3072), ("nn", 6304, 3072, 768),
    ("tn", 2304, 768, 6304), ("tn", 3072, 768, 6304), ("tn", 768, 3072, 6304),
    ("nt", 2048, 2304, 768), ("nt", 2048, 3072, 768), ("nt", 2048, 768, 3072), ("nn", 2048, 768, 3072),
    ("tn", 3072, 768, 2048), ("nt", 2048, 50256, 768),
]
TILES = [int(t) for t in os.environ.get("GEMM_TILES", "0,1,2,5,6,7,8,9,10,11,12").split(",")]
if os.environ.get("GEMM_SHAPES"):  # "nt:M:N:K,nn:M:N:K,..."
    SHAPES = [(f.split(":")[0],) + tuple(int(v) for v in f.split(":")[1:]) for f in os.environ["GEMM_SHAPES"].split(",")]
if "--big" in sys.argv:
    SHAPES = [("nt", 8192, 8192, 8192), ("nt", 4096, 4096, 4096)] + SHAPES

for lay, M, N, K in SHAPES:
    a_tr, b_tr = lay[0] == "t", lay[1] == "n"
    a = torch.randn(K, M, device="cuda").bfloat16() if a_tr else torch.randn(M, K, device="cuda").bfloat16()
    b = (torch.randn(K, N, device="cuda") if b_tr else torch.randn(N, K, device="cuda")).bfloat16() * 0.05
    av = a.t() if a_tr else a
    bv = b if b_tr else b.t()
    flop = 2.0 * M * N * K
    row = {"layout": lay, "M": M, "N": N, "K": K, "vendor_us": round(t_us(lambda: av @ bv), 1)}
    best = (1e30, None)
    for t in TILES:
        for sp in (1, 2, 3, 4, 6):
            if sp > 1 and K // sp < 256:
                continue
            try:
                us = t_us(lambda: C.gemm(a, b, a_tr=a_tr, b_tr=b_tr, tile=t, splits=sp))
            except RuntimeError:
                continue
            row[f"t{t}s{sp}"] = round(us, 1)
            if us < best[0]:
                best = (us, f"t{t}s{sp}")
    row["best"] = best[1]
    row["best_us"] = round(best[0], 1)
    row["best_tf"] = round(flop / best[0] / 1e6, 0)
    row["vendor_tf"] = round(flop / row["vendor_us"] / 1e6, 0)
    row["native_over_vendor"] = round(row["vendor_us"] / best[0], 3)
    print(json.dumps(row), flush=True)
