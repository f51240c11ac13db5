"""Debug: deferred weight-gradient reduce — which gradients differ, and were they stolen by AccumulateGrad?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hyperion.ops.conv as hconv  # noqa: E402
from hyperion.models.resnet import Bottleneck  # noqa: E402
from hyperion.train.amp import cast_for_compute  # noqa: E402

torch.manual_seed(0)
m = Bottleneck(256, 64).cuda().to(memory_format=torch.channels_last)
cast_for_compute(m, torch.bfloat16)
x0 = torch.randn(8, 256, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
gy = torch.randn(8, 256, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
orig = hconv._wgrad
made = {}


def spy(dy, x, w, stride, padding, w_param=None):
    dw = orig(dy, x, w, stride, padding, w_param=w_param)
    made[id(w_param) if w_param is not None else id(w)] = (dw.data_ptr(), tuple(dw.stride()), w_param is not None,
                                                           hconv._defer_state["pending"])
    return dw


hconv._wgrad = spy
for name, p in m.named_parameters():
    print(name, tuple(p.shape), tuple(p.stride()), p.is_leaf, p.dtype)


def run(defer):
    hconv.DEFER_WGRAD_REDUCE = defer
    made.clear()
    for p in m.parameters():
        p.grad = None
    m(x0.clone().requires_grad_(True)).backward(gy)
    torch.cuda.synchronize()
    out = {}
    for n, p in m.named_parameters():
        info = made.get(id(p))
        out[n] = (p.grad.float().clone(), info, p.grad.data_ptr(), tuple(p.grad.stride()))
    return out


a = run(False)
b = run(True)
for n in a:
    ga, ia, pa, sa = a[n]
    gb, ib, pb, sb = b[n]
    print(n, "equal" if torch.equal(ga, gb) else f"DIFF max {(ga - gb).abs().max().item():.3e}",
          "| defer-run dw info", ib, "grad ptr", pb, "stride", sb, "stolen" if ib and ib[0] == pb else "not-stolen")
