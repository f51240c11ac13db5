"""fp32 GEMM tile shapes (gemm_f32.hip: 0 128x128, 1 256x64, 2 64x256, 3 256x128, 4 128x256) at one
split vs hipBLASLt, NT layout: one JSON line per GEMM shape."""
import json
import sys

import torch

sys.path.insert(0, ".")
from hyperion.ops import _native  # noqa: E402
from hyperion.ops.gemm import _time  # noqa: E402

C = _native.native()
for M, N, K in [(8192, 8192, 8192), (4096, 4096, 4096), (6304, 2304, 768), (6304, 768, 3072), (6304, 3072, 768),
                (100352, 64, 576), (25088, 128, 1152), (6272, 256, 2304), (1568, 512, 4608)]:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda")
    reps = 3 if M * N * K > 1e11 else 10
    r = {"M": M, "N": N, "K": K, "vendor_us": round(_time(lambda: a @ b.t(), reps) / reps * 1e3, 1)}
    for shape in range(5):
        for sp in (1, 2, 4):
            try:
                r[f"s{shape}x{sp}"] = round(_time(lambda: C.gemm_f32(a, b, shape=shape, splits=sp), reps) / reps * 1e3, 1)
            except RuntimeError:
                pass
    best = min((v, k) for k, v in r.items() if k.startswith("s"))
    r["best"], r["best_tf"], r["vendor_tf"] = best[1], round(2 * M * N * K / best[0] / 1e6, 1), round(2 * M * N * K / r["vendor_us"] / 1e6, 1)
    print(json.dumps(r), flush=True)
