"""hipGraph-captured training step == eager step (ResNet-18, native conv/BN kernels + fused Adam)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graph: bool, steps: int):
    from hyperion.models import resnet18
    from hyperion.ops import FusedAdam
    from hyperion.train.amp import cast_for_compute
    from hyperion.train.step import TrainStep

    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    cast_for_compute(model, torch.bfloat16)
    init = [p.detach().float().clone() for p in model.parameters()]
    # eps=1: update ~ lr*m (linear in the gradient), so vendor-kernel nondeterminism is not
    # amplified into +-lr sign steps the way Adam does it for near-zero gradients
    opt = FusedAdam(model.parameters(), lr=1e-2, eps=1.0)
    step = TrainStep(model, opt, torch.nn.MSELoss(), amp_dtype=None, graph=graph, warmup_iters=2)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(8, 3, 64, 64, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.rand(8, 10, device=dev, generator=g)
    losses = [float(step(x, y)) for _ in range(steps)]
    torch.cuda.synchronize()
    delta = [p.detach().float() - i for p, i in zip(model.parameters(), init)]
    return losses, delta


def _dist(a, b):
    return sum(float((u - v).norm() ** 2) for u, v in zip(a, b)) ** 0.5


def test_graph_step_matches_eager():
    # the graph path runs `warmup_iters` eager warm-up steps before capture: 2 + 4 = 6 updates
    le, de = _run(False, steps=6)
    le2, de2 = _run(False, steps=6)  # run-to-run noise of the eager path itself
    lg, dg = _run(True, steps=4)
    assert all(torch.isfinite(torch.tensor(lg)))
    torch.testing.assert_close(torch.tensor(lg[-1]), torch.tensor(le[-1]), rtol=3e-2, atol=3e-3)
    ref = sum(float(a.norm() ** 2) for a in de) ** 0.5
    noise = _dist(de, de2)
    assert ref > 0 and _dist(de, dg) <= 2.0 * noise + 0.03 * ref, (_dist(de, dg), noise, ref)
