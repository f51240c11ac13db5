"""hipGraph-captured training step == eager step (ResNet-18, native BN + fused Adam)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graph: bool, steps: int = 4):
    from hyperion.models import resnet18
    from hyperion.ops import FusedAdam
    from hyperion.train.amp import cast_for_compute
    from hyperion.train.step import TrainStep

    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    cast_for_compute(model, torch.bfloat16)
    opt = FusedAdam(model.parameters(), lr=1e-3)
    step = TrainStep(model, opt, torch.nn.MSELoss(), amp_dtype=None, graph=graph, warmup_iters=2)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(8, 3, 64, 64, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.rand(8, 10, device=dev, generator=g)
    losses = [float(step(x, y)) for _ in range(steps)]
    torch.cuda.synchronize()
    return losses, [p.detach().float().clone() for p in model.parameters()]


def test_graph_step_matches_eager():
    # the graph path runs `warmup_iters` eager warm-up steps before capture; compare trajectories
    # after the same number of optimizer updates
    le, pe = _run(False, steps=6)
    lg, pg = _run(True, steps=4)  # 2 warm-up + 4 replays = 6 updates
    assert all(torch.isfinite(torch.tensor(lg)))
    torch.testing.assert_close(torch.tensor(lg[-1]), torch.tensor(le[-1]), rtol=2e-2, atol=2e-3)
    # MIOpen's wgrad is not bitwise deterministic and Adam turns sign flips of near-zero grads into
    # +-lr steps, so compare parameters by relative norm, not elementwise
    for a, b in zip(pe, pg):
        assert (a - b).norm() <= 0.05 * a.norm() + 1e-3
