"""Timed fp32 training steps (reference methodology model, Adam, MSE) for kernel traces:
``python scripts/fp32_step.py <model> <native 0|1> [steps]``."""
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from hyperion.bench.baseline import baseline_suite  # noqa: E402
from hyperion.ops import conv_f32  # noqa: E402

name, native = sys.argv[1], sys.argv[2] == "1"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
conv_f32.ENABLED = native
fn, ishape, tshape = next((f, i, t) for n, f, i, t in baseline_suite(real_vit=True) if n == name)
m = fn().cuda().to(memory_format=torch.channels_last)
opt = torch.optim.Adam(m.parameters(), lr=1e-3)
x = torch.randn(*ishape, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.rand(*tshape, device="cuda")
for i in range(steps + 3):
    if i == 3:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    F.mse_loss(m(x), y).backward()
    opt.step()
torch.cuda.synchronize()
print(f"{name} native={native} {1e3 * (time.perf_counter() - t0) / steps:.3f} ms/step")
if native:
    print("routes (native faster):", sum(conv_f32._ROUTE.values()), "of", len(conv_f32._ROUTE))
    for k, v in conv_f32._ROUTE.items():
        tn, tv = conv_f32.ROUTE_MS.get(k, (0.0, 0.0))
        print("  ", k[0], k[1], k[2], k[3], "native" if v else "vendor", f"native {tn * 1e3:.1f} us vendor {tv * 1e3:.1f} us")
