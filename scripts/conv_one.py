"""Run one ResNet-50 conv shape (fwd with BN stats, dgrad, wgrad) a few times — PMC counter target."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

N, C, H, K, R, s, p = [int(v) for v in (sys.argv[1:8] if len(sys.argv) > 7 else (32, 256, 14, 256, 3, 1, 1))]
C_ = _native.native()
x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
P = (H + 2 * p - R) // s + 1
dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for _ in range(10):
    C_.conv_fwd(x, w, s, s, p, p, True)
    if s == 1:
        C_.conv_dgrad(dy, w, p, p)
    C_.conv_wgrad(dy, x, R, R, s, s, p, p)
torch.cuda.synchronize()
print("ok")
