"""Diagnose write-through store results: small-M BN backward (bn_bwd_small_k) and the conv_bn_act
test case, each checked against torch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C_ = _native.native()
torch.manual_seed(0)
for M_img, Cc, res in [(2 * 14 * 14, 64, True), (2 * 14 * 14, 64, False), (8 * 28 * 28, 128, True)]:
    N = 2
    H = int((M_img / N) ** 0.5)
    x = torch.randn(N, Cc, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    w = torch.rand(Cc, device="cuda") + 0.5
    b = torch.randn(Cc, device="cuda") * 0.1
    xf = x.float()
    mean = xf.mean((0, 2, 3))
    var = xf.var((0, 2, 3), unbiased=False)
    invstd = torch.rsqrt(var + 1e-5)
    y = torch.relu((xf - mean.view(1, -1, 1, 1)) * (invstd * w).view(1, -1, 1, 1) + b.view(1, -1, 1, 1))
    yb = y.bfloat16().contiguous(memory_format=torch.channels_last)
    sums = torch.zeros(_native.STAT_SLOTS * 2 * Cc, device="cuda", dtype=torch.float64)
    dx, dres, dw, db = C_.bn_bwd(dy, x, yb, w, b, mean, invstd, True, True, res, sums=sums)
    torch.cuda.synchronize()
    # reference
    xr = xf.detach().cpu().requires_grad_(True)
    wr = w.cpu().requires_grad_(True)
    br = b.cpu().requires_grad_(True)
    out = torch.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5))
    out.backward(dy.float().cpu())
    err = (dx.float().cpu() - xr.grad).norm() / xr.grad.norm()
    print(f"bn_bwd M={x.numel() // Cc} C={Cc} res={res}: dx finite={bool(torch.isfinite(dx).all())} rel={err.item():.3e}"
          + (f" dres finite={bool(torch.isfinite(dres).all())}" if res else ""))
