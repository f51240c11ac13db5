"""One attention shape, fwd + bwd a few times (for rocprofv3 --pmc passes):
python scripts/attn_one.py B S H D causal(0/1)"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

B, S, H, D, causal = (int(v) for v in sys.argv[1:6])
C = _native.native()
q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(4))
scale = 1.0 / math.sqrt(D)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(3):
    o, lse = C.attn_fwd(q, k, v, bool(causal), scale, 0.0, None, None, True)
    C.attn_bwd(do, q, k, v, o, lse, bool(causal), scale, 0.0, None, None, dq, dk, dv)
torch.cuda.synchronize()
print("ok", flush=True)
