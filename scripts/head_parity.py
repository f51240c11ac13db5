"""Per-step loss of the bench's ResNet-50 step with the fused head (--loss head) vs torch fc + MSE,
from identical weights and data (eager and hipGraph).  Usage: python scripts/head_parity.py"""
import json
import sys

import torch
import torch.nn as nn

sys.path.insert(0, ".")
import hyperion  # noqa: F401,E402
from hyperion.models import resnet50  # noqa: E402
from hyperion.ops import FusedAdam  # noqa: E402
from hyperion.ops.losses import LinearMSELoss  # noqa: E402
from hyperion.train.amp import cast_for_compute  # noqa: E402
from hyperion.train.step import TrainStep  # noqa: E402


def run(head: bool, graph: bool, steps: int = 12):
    torch.manual_seed(1234)
    dev = torch.device("cuda")
    model = resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
    cast_for_compute(model, torch.bfloat16)
    opt = FusedAdam(model.parameters(), lr=1e-3, zero_grad_in_step=True)
    loss_fn = nn.MSELoss()
    if head:
        model.head_in_loss = True
        loss_fn = LinearMSELoss(model.fc)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.rand(32, 3, 224, 224, device=dev, generator=g).to(memory_format=torch.channels_last).to(torch.bfloat16)
    y = torch.rand(32, 1000, device=dev, generator=g)
    step = TrainStep(model, opt, loss_fn, amp_dtype=None, graph=graph)
    return [round(float(step(x, y).float().item()), 6) for _ in range(steps)]


for graph in (False, True):
    a, b = run(False, graph), run(True, graph)
    print(json.dumps({"graph": graph, "torch_fc_mse": a, "fused_head": b,
                      "max_rel_diff": max(abs(p - q) / abs(p) for p, q in zip(a, b))}), flush=True)
