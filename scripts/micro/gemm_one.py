"""One native GEMM shape, repeated (for rocprofv3 PMC passes): python scripts/micro/gemm_one.py M N K tile splits [vendor]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from hyperion.ops import _native  # noqa: E402

M, N, K, tile, splits = (int(v) for v in sys.argv[1:6])
vendor = len(sys.argv) > 6 and sys.argv[6] == "vendor"
C = _native.native()
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
for _ in range(30):
    y = x @ w.t() if vendor else C.gemm(x, w, tile=tile, splits=splits)
torch.cuda.synchronize()
print("ok", tuple(y.shape))
