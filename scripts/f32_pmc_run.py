"""One fp32 GEMM shape run a few times (for a rocprofv3 --pmc pass): python scripts/f32_pmc_run.py M N K"""
import sys

import torch

sys.path.insert(0, ".")
from hyperion.ops import _native  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
a = torch.randn(M, K, device="cuda")
b = torch.randn(N, K, device="cuda")
C = _native.native()
for _ in range(5):
    C.gemm_f32(a, b, shape=0, splits=1)
torch.cuda.synchronize()
