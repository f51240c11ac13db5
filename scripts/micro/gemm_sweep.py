"""Time one NT GEMM shape on every native tile (split 1) and on the vendor GEMM, HBM-warm and with
a 512 MiB scrub between calls (HBM-cold):  python scripts/micro/gemm_sweep.py M N K [M N K ...]"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from hyperion.ops import _native  # noqa: E402

C = _native.native()
args = [int(v) for v in sys.argv[1:]]
scrub = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")


def t_us(fn, cold, reps=10):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    for s, e in ev:
        if cold:
            scrub.add_(1)
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return sorted(s.elapsed_time(e) for s, e in ev)[reps // 2] * 1e3


for i in range(0, len(args), 3):
    M, N, K = args[i:i + 3]
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    flop = 2.0 * M * N * K
    row = {"M": M, "N": N, "K": K}
    for name, fn in [("vendor", lambda: x @ w.t())] + [
            (f"t{t}", (lambda t=t: C.gemm(x, w, tile=t, splits=1))) for t in (0, 1, 2, 4, 5, 6, 7)]:
        try:
            warm, cold = t_us(fn, False), t_us(fn, True)
        except RuntimeError as e:
            row[name] = str(e)[:40]
            continue
        row[name] = {"warm_us": round(warm, 1), "cold_us": round(cold, 1), "warm_tf": round(flop / warm / 1e6, 0)}
    print(json.dumps(row), flush=True)

# weight-gradient (TN) shapes: env GEMM_TN="N K T,..." (dy [T, N], x [T, K] -> [N, K]), tiles 1 / 8 / 0 / 2
import os  # noqa: E402

for spec in [s for s in os.environ.get("GEMM_TN", "").split(",") if s.strip()]:
    N, K, T = (int(v) for v in spec.split())
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    flop = 2.0 * N * K * T
    row = {"tn": [N, K, T], "vendor": round(t_us(lambda: dy.t() @ x, False), 1)}
    for t in (0, 1, 2):
        for sp in (1, 2, 3, 4, 6, 8):
            try:
                us = t_us(lambda: C.gemm(dy, x, a_tr=True, b_tr=True, tile=t, splits=sp), False)
            except RuntimeError:
                continue
            row[f"t{t}s{sp}"] = round(us, 1)
    best = min((v, k) for k, v in row.items() if k.startswith("t") and k != "tn")
    row["best"] = best[1]
    row["best_tf"] = round(flop / best[0] / 1e6, 0)
    print(json.dumps(row), flush=True)
