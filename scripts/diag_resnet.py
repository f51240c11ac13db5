"""Diagnose native-vs-torch divergence of a whole ResNet (forward per block, then grads)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hyperion.models.resnet import resnet18, resnet50  # noqa: E402
from hyperion.ops import _native  # noqa: E402
from hyperion.train.amp import cast_for_compute  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
torch.manual_seed(0)
m32 = (resnet50 if arch == "resnet50" else resnet18)(num_classes=16).cuda().to(memory_format=torch.channels_last)
m = copy.deepcopy(m32)
cast_for_compute(m, torch.bfloat16)
x0 = torch.randn(4, 3, 96, 96, device="cuda").contiguous(memory_format=torch.channels_last)
gy = torch.randn(4, 16, device="cuda")

acts = {}


def hook(tag):
    def f(mod, inp, out):
        acts.setdefault(tag, []).append(out.detach().float())
    return f


for name, mod in list(m.named_children()) + [("layer1.0", m.layer1[0])]:
    mod.register_forward_hook(hook("bf16:" + name))
for name, mod in list(m32.named_children()) + [("layer1.0", m32.layer1[0])]:
    mod.register_forward_hook(hook("fp32:" + name))


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


x = x0.bfloat16().requires_grad_(True)
m(x).float().backward(gy)
g_native = [p.grad.float().clone() for p in m.parameters()]
dx_native = x.grad.float().clone()
fwd_native = {k: v[0] for k, v in acts.items()}
acts.clear()
os.environ["HYPERION_KERNELS"] = "torch"
for p in m.parameters():
    p.grad = None
x2 = x0.bfloat16().requires_grad_(True)
m(x2).float().backward(gy)
g_torch16 = [p.grad.float().clone() for p in m.parameters()]
fwd_torch16 = {k: v[0] for k, v in acts.items()}
acts.clear()
xr = x0.clone().requires_grad_(True)
m32(xr).backward(gy)
fwd32 = {k: v[0] for k, v in acts.items()}
for name, _ in list(m.named_children()) + [("layer1.0", None)]:
    a, t, b = fwd_native.get("bf16:" + name), fwd_torch16.get("bf16:" + name), fwd32.get("fp32:" + name)
    if a is not None and b is not None:
        print(f"fwd {name:10s} native-vs-fp32 {rel(a, b):.3e}  torchbf16-vs-fp32 {rel(t, b):.3e}  native-vs-torchbf16 {rel(a, t):.3e}")
print(f"dx native-vs-fp32 {rel(dx_native, xr.grad):.3e} torchbf16-vs-fp32 {rel(x2.grad.float(), xr.grad):.3e}")
for (n, p), gn, gt, p32 in zip(m.named_parameters(), g_native, g_torch16, m32.parameters()):
    print(f"grad {n:36s} native-fp32 {rel(gn, p32.grad):.3e} torch16-fp32 {rel(gt, p32.grad):.3e} native-torch16 {rel(gn, gt):.3e}")
