"""ResNet-50 stem (7x7/s2/p3, 3->64, batch 32, 224², bf16) piece by piece: Hyperion's space-to-depth
path (stem.hip + conv kernels with a 16-element pixel stride) vs MIOpen (F.conv2d /
convolution_backward), hipGraph-timed (20 launches per graph)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from hyperion.ops import _native  # noqa: E402
from hyperion.ops.conv import stem_weight, stem_weight_grad  # noqa: E402
from conv_roofline import gtime  # noqa: E402

C_ = _native.native()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
x = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
xs = C_.stem_s2d(x)
w4 = stem_weight(w)
sums = torch.zeros(_native.STAT_SLOTS * 2 * 64, device="cuda", dtype=torch.float64)
y = C_.stem_conv_fwd(xs, w4, sums)
dy = torch.randn_like(y)
r = {"s2d_us": gtime(lambda: C_.stem_s2d(x)), "w4_us": gtime(lambda: stem_weight(w)),
     "fwd_us": gtime(lambda: C_.stem_conv_fwd(xs, w4, sums))}
for sp in (-1, 64, 128, 256, 512, 1024):
    r[f"wgrad_s{sp}_us"] = gtime(lambda: C_.stem_conv_wgrad(dy, xs, sp))
dw4 = C_.stem_conv_wgrad(dy, xs)
r["dw_us"] = gtime(lambda: stem_weight_grad(dw4, 3))
r["miopen_fwd_us"] = gtime(lambda: F.conv2d(x, w, None, 2, 3))
r["miopen_wgrad_us"] = gtime(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False,
                                                                          [0, 0], 1, [False, True, False]))
print(json.dumps({k: round(v, 2) for k, v in r.items()}))
