"""fp32 GEMM: native fp32-MFMA kernel (cost-model plan and tuned plan) vs torch.mm (hipBLASLt) on the
fp32 linear shapes of the reference-methodology models (ViT-B/16 b32, CustomTransformer, LM-768)
and the C3 square sizes.  One JSON line per (shape, layout)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from hyperion.ops import _native, conv_f32  # noqa: E402
from hyperion.ops.gemm import _time  # noqa: E402

C = _native.native()
SHAPES = [(6304, 2304, 768), (6304, 768, 3072), (8192, 8192, 8192), (4064, 3072, 768)] if "--short" in sys.argv else [(6304, 2304, 768), (6304, 768, 768), (6304, 3072, 768), (6304, 768, 3072), (4096, 4096, 4096),
          (8192, 8192, 8192), (512, 2048, 512), (512, 512, 2048), (4064, 768, 768), (4064, 3072, 768)]
for M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda")
    for lay in ("nt", "nn", "tn"):
        if lay == "nt":
            A, B, at, bt, ven = a, b, False, False, (lambda: a @ b.t())
        elif lay == "nn":
            bb = b.t().contiguous()  # [K, N]: B(n, k) = bb[k, n]
            A, B, at, bt, ven = a, bb, False, True, (lambda: a @ bb)
        else:
            aa = a.t().contiguous()
            bb = b.t().contiguous()
            A, B, at, bt, ven = aa, bb, True, True, (lambda: aa.t() @ bb)
        reps = 3 if M * N * K > 2e11 else 10
        tv = _time(ven, reps) / reps * 1e3
        tm = _time(lambda: C.gemm_f32(A, B, a_tr=at, b_tr=bt), reps) / reps * 1e3
        conv_f32._PLAN.clear()
        conv_f32.gemm(A, B, at, bt)
        tt = _time(lambda: conv_f32.gemm(A, B, at, bt), reps) / reps * 1e3
        fl = 2.0 * M * N * K
        print(json.dumps({"M": M, "N": N, "K": K, "layout": lay, "vendor_us": round(tv, 1), "model_us": round(tm, 1),
                          "tuned_us": round(tt, 1), "plan": list(conv_f32._PLAN.values())[0],
                          "vendor_tf": round(fl / tv / 1e6, 1), "tuned_tf": round(fl / tt / 1e6, 1)}), flush=True)
