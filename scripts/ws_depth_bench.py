"""Weight-streaming GEMM at 4 vs 8 k-steps in flight per wave (ws_set_depth), Llama-2-7B shapes at
M = 128, HBM-cold weights (ws_bench.py's pool timing).  python scripts/ws_depth_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C = _native.native()


def timed(fn, pool, reps=3):
    import statistics
    for w in pool[:2]:
        fn(w)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for w in pool:
            fn(w)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / len(pool))
    return statistics.median(ts)


rows = []
for name, N, K in [("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008)]:
    n = max(3, -(-(640 << 20) // (N * K * 2)))
    pool = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(n)]
    x = torch.randn(128, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(128, N, device="cuda", dtype=torch.bfloat16)
    r = {"name": name}
    for d in (4, 8):
        C.ws_set_depth(d)
        r[f"nt_d{d}"] = round(timed(lambda w: C.ws_gemm_part(x, w, slab16=True), pool), 2)
        r[f"nn_d{d}"] = round(timed(lambda w: C.ws_gemm_part(dy, w, nn=True, slab16=True), pool), 2)
        r[f"nt_d{d}_TBs"] = round(N * K * 2 / r[f"nt_d{d}"] / 1e6, 2)
        r[f"nn_d{d}_TBs"] = round(N * K * 2 / r[f"nn_d{d}"] / 1e6, 2)
    C.ws_set_depth(4)
    print(json.dumps(r), flush=True)
    rows.append(r)
    del pool
    torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(rows, open("gpurun_out/ws_depth_bench.json", "w"), indent=1)
