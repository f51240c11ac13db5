"""Sweep split count / tile width / LDS stages of the skinny linear kernels on Llama-2-7B shapes."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C = _native.native()


def med(fn, rep=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(rep):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


out = []
for (M, K, N) in [(128, 4096, 4096), (128, 4096, 11008), (128, 11008, 4096)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    wbytes = N * K * 2
    r = {"M": M, "K": K, "N": N, "hipblaslt_nt": med(lambda: torch.nn.functional.linear(x, w)),
         "hipblaslt_nn": med(lambda: dy @ w)}
    for nb in (2, 3, 4):
        C.conv_set_stages(nb, 0)
        for bn in (64, 128):
            for sp in (1, 2, 4, 6, 8, 12, 16):
                r[f"nt_nb{nb}_bn{bn}_sp{sp}"] = med(lambda: C.linear_nt(x, w, sp, bn))
                r[f"nn_nb{nb}_bn{bn}_sp{sp}"] = med(lambda: C.linear_nn(dy, w, sp, bn))
    C.conv_set_stages(0, 0)
    r["nt_auto"] = med(lambda: C.linear_nt(x, w))
    r["nn_auto"] = med(lambda: C.linear_nn(dy, w))
    for kind in ("nt", "nn"):
        best = min((v, k) for k, v in r.items() if k.startswith(kind + "_nb"))
        r[f"{kind}_best"] = best
        print(M, K, N, kind, "best", best, "auto", r[f"{kind}_auto"], "hipblaslt", r[f"hipblaslt_{kind}"],
              f"best TB/s {wbytes / best[0] / 1e6:.2f}", flush=True)
    out.append(r)
json.dump(out, open("gpurun_out/skinny_sweep.json", "w"), indent=1)
