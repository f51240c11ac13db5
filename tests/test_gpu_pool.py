"""NHWC pooling kernels (pool.hip) vs PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 112, 112), 3, 2, 1), ((2, 128, 56, 56), 3, 2, 1),
                                         ((3, 16, 9, 11), 2, 2, 0), ((2, 8, 7, 7), 3, 1, 1),
                                         ((3, 16, 9, 11), 3, 2, 0), ((2, 8, 13, 15), 3, 2, 1)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool_fwd_bwd_match_torch(shape, k, s, p, dtype):
    from hyperion.ops.pool import max_pool2d

    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = max_pool2d(x, k, s, p)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().cpu().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    yr.backward(g.float().cpu())
    torch.testing.assert_close(y.float().cpu(), yr)
    torch.testing.assert_close(x.grad.float().cpu(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("shape", [(32, 2048, 7, 7), (5, 64, 3, 4)])
def test_global_avgpool_fwd_bwd(shape):
    from hyperion.ops.pool import global_avg_pool

    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = global_avg_pool(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    yr = F.adaptive_avg_pool2d(xr, 1)
    yr.backward(g.float())
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-3)
