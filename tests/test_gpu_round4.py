"""Round-4 native paths vs plain fp32 PyTorch references.

* the ResNet RGB stem (7x7/s2/p3, C=3) on the native conv kernels: ``stem.hip`` space-to-depth
  (exact copy of the torch reference rewrite), then conv_fwd / conv_wgrad as a stride-1 R=4 conv
  with a 16-element pixel stride — forward, BN statistics and weight gradient against fp32
  ``F.conv2d`` + BN + ReLU (reference stem: torchvision ResNet conv1 on MIOpen,
  ``Phase 1/baseline_performance.ipynb:203-205``).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 3, 224, 224), (3, 3, 33, 31), (1, 4, 17, 18), (2, 1, 64, 64)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_stem_s2d_kernel_is_the_reference_rewrite(shape, dtype):
    from hyperion.ops import _native
    from hyperion.ops.conv import stem_s2d_reference

    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    got = _native.native().stem_s2d(x)
    ref = stem_s2d_reference(x)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, ref)  # a pure gather: bit-exact


@pytest.mark.parametrize("N,H", [(4, 64), (2, 224)])
def test_stem_conv_bn_relu_native_matches_fp32(N, H):
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act

    torch.manual_seed(0)
    _native.reset_counters()
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda()
    bn = BatchNormAct2d(64, act=True).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    conv_l = conv.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(N, 3, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out = conv_bn_act(conv_l, bn, x)
    g = torch.randn_like(out)
    out.backward(g)
    cnt = _native.counters()
    assert cnt.get("stem_s2d") == 1 and cnt.get("conv_bn_act") == 1 and "conv_bn_act_fallback" not in cnt, cnt
    assert cnt.get("wgrad") == 1 and "wgrad_vendor" not in cnt, cnt
    wr = conv_l.weight.detach().float().cpu().requires_grad_(True)
    y = F.conv2d(x.float().cpu(), wr, stride=2, padding=3)
    y = F.relu(F.batch_norm(y, None, None, bn.weight.detach().cpu(), bn.bias.detach().cpu(), True, 0.1, bn.eps))
    y.backward(g.float().cpu())
    torch.testing.assert_close(out.float().cpu(), y.detach(), rtol=3e-2, atol=3e-2)
    dw = conv_l.weight.grad.float().cpu()
    assert dw.shape == wr.grad.shape
    torch.testing.assert_close(dw, wr.grad, rtol=3e-2, atol=3e-2 * wr.grad.abs().max().item())
