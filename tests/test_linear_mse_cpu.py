"""LinearMSELoss / ResNet head_in_loss wiring on CPU (the torch fallback of ops.losses.linear_mse)."""
import torch
import torch.nn.functional as F


def test_head_in_loss_matches_model_fc_and_mse():
    from hyperion.models import resnet18
    from hyperion.ops.losses import LinearMSELoss

    torch.manual_seed(0)
    model = resnet18(num_classes=10)
    x = torch.randn(2, 3, 32, 32)
    y = torch.rand(2, 10)
    ref = F.mse_loss(model(x), y)
    ref.backward()
    gref = model.fc.weight.grad.clone()
    model.zero_grad(set_to_none=True)

    model.head_in_loss = True
    loss_fn = LinearMSELoss(model.fc)
    assert not list(loss_fn.parameters()), "the loss must not re-register the model's head"
    feats = model(x)
    assert feats.shape == (2, 512)
    loss = loss_fn(feats, y)
    loss.backward()
    assert torch.allclose(loss, ref, rtol=1e-5, atol=1e-6)
    assert torch.allclose(model.fc.weight.grad, gref, rtol=1e-5, atol=1e-6)
