"""Fused classifier head + MSE (linear_mse.hip) vs a plain fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # M, K, N
    (32, 2048, 1000),  # the ResNet-50 step benchmark head
    (5, 64, 37),       # ragged N, a partial column tile, few rows
    (64, 520, 130),    # M at the cap, K not a multiple of the 128-deep chunk
]


def _reference(x, w, b, y, scale):
    xf, wf = x.float().clone().requires_grad_(), w.float().clone().requires_grad_()
    bf = b.float().clone().requires_grad_() if b is not None else None
    z = F.linear(xf, wf, bf).to(x.dtype).float()  # logits in the compute dtype, as the unfused head
    loss = F.mse_loss(z, y)
    (loss * scale).backward()
    return loss.detach(), xf.grad, wf.grad, (bf.grad if bf is not None else None)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("bias", [True, False])
def test_linear_mse_matches_fp32(shape, dtype, bias):
    from hyperion.ops import _native
    from hyperion.ops.losses import linear_mse

    M, K, N = shape
    torch.manual_seed(0)
    dev = torch.device("cuda")
    x = torch.randn(M, K, device=dev).to(dtype)
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dtype)
    b = (torch.randn(N, device=dev) * 0.1).to(dtype) if bias else None
    y = torch.rand(M, N, device=dev)
    ref_loss, rdx, rdw, rdb = _reference(x, w, b, y, 3.0)

    xs, ws = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    bs = b.detach().clone().requires_grad_() if bias else None
    before = _native.counters().get("linear_mse", 0)
    loss = linear_mse(xs, ws, bs, y)
    assert _native.counters().get("linear_mse", 0) == before + 1, "native linear_mse path did not run"
    (loss * 3.0).backward()
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert torch.allclose(loss.float(), ref_loss, rtol=1e-3 if dtype == torch.bfloat16 else 1e-5, atol=1e-6)
    for got, ref in ((xs.grad, rdx), (ws.grad, rdw)) + (((bs.grad, rdb),) if bias else ()):
        assert got.dtype == dtype
        err = (got.float() - ref).abs().max().item()
        assert err <= tol * ref.abs().max().item() + 1e-6, err


def test_linear_mse_graph_replay_deterministic():
    """The last-arriver ticket resets itself: replays of a captured step give bit-identical results."""
    from hyperion.ops.losses import linear_mse

    torch.manual_seed(1)
    dev = torch.device("cuda")
    x = torch.randn(32, 2048, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(1000, 2048, device=dev) * 0.02).to(torch.bfloat16).requires_grad_()
    b = torch.zeros(1000, device=dev, dtype=torch.bfloat16, requires_grad=True)
    y = torch.rand(32, 1000, device=dev)

    def step():
        x.grad = w.grad = b.grad = None
        loss = linear_mse(x, w, b, y)
        loss.backward()
        return loss

    eager = step().detach().clone()
    g_eager = w.grad.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    x.grad = w.grad = b.grad = None
    with torch.cuda.graph(g):
        out = linear_mse(x, w, b, y)
        out.backward()
    outs = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        outs.append(out.clone())
        assert torch.equal(w.grad, g_eager)
    assert all(torch.equal(o, eager) for o in outs)


def test_resnet_head_in_loss_matches_unfused():
    """ResNet-18 with head_in_loss + LinearMSELoss == the model's own fc + nn.MSELoss."""
    from hyperion.models import resnet18
    from hyperion.ops.losses import LinearMSELoss

    torch.manual_seed(2)
    dev = torch.device("cuda")
    model = resnet18(num_classes=100).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device=dev).to(memory_format=torch.channels_last)
    y = torch.rand(4, 100, device=dev)
    ref = F.mse_loss(model(x).float(), y)
    ref.backward()
    gref = model.fc.weight.grad.clone()
    model.zero_grad(set_to_none=True)
    model.head_in_loss = True
    loss_fn = LinearMSELoss(model.fc)
    feats = model(x)
    assert feats.shape == (4, 512)
    loss = loss_fn(feats, y)
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 1e-3 * abs(ref.item()) + 1e-5
    assert torch.allclose(model.fc.weight.grad, gref, rtol=1e-3, atol=1e-5)
