"""BN apply + ReLU fused into the consuming conv's operand read (``conv_igemm.hip`` XF mode).

The consumer conv reads the producer's RAW conv output, finalizes the producer's BatchNorm
statistics inline and computes with ``relu(x * scale + shift)`` — against the unfused pipeline
(``bn_fwd_sums`` apply pass, then the conv on the materialized activation) every result must be
bit-identical: the conv output, the side-written activation, save_mean / save_invstd and the
running statistics (same bf16 operands, same fp32 / fp64 arithmetic).  Then a ResNet-50 training
step with the fusion on vs off (``ops/conv.py`` FUSE_BN_APPLY).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sums_of(y: torch.Tensor, slots: int) -> torch.Tensor:
    C = y.shape[1]
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, C).double()
    s = torch.zeros(slots, 2, C, device=y.device, dtype=torch.float64)
    s[0, 0] = yf.sum(0)
    s[0, 1] = (yf * yf).sum(0)
    return s.reshape(-1).contiguous()


@pytest.mark.parametrize("shape", [(4, 64, 28, 256, 1, 0), (2, 64, 14, 64, 3, 1), (2, 512, 7, 512, 3, 1),
                                   (3, 128, 9, 128, 3, 1), (2, 256, 14, 1024, 1, 0), (4, 256, 4, 256, 3, 1),
                                   (4, 512, 2, 512, 3, 1), (4, 512, 2, 2048, 1, 0)])
@pytest.mark.parametrize("tile", [(64, 64), (128, 64), (128, 128)])
@pytest.mark.parametrize("splits,stages", [(1, 2), (1, 1), (1, 3), (3, 2)])
def test_conv_xf_matches_apply_then_conv_bitwise(shape, tile, splits, stages):
    from hyperion.ops import _native

    C = _native.native()
    N, Cin, H, K, R, p = shape
    torch.manual_seed(0)
    y0 = (torch.randn(N, Cin, H, H, device="cuda") * 2 + 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, Cin, R, R, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    g = torch.randn(Cin, device="cuda")  # some negative BN weights: the padding must still read 0
    b = torch.randn(Cin, device="cuda") * 0.5
    sums = _sums_of(y0, _native.STAT_SLOTS)
    rm0, rv0 = torch.randn(Cin, device="cuda"), torch.rand(Cin, device="cuda") + 0.5

    rmA, rvA = rm0.clone(), rv0.clone()
    a, mean, invstd = C.bn_fwd_sums(y0, None, sums, g, b, rmA, rvA, 0.1, 1e-5, True)
    sA = torch.zeros(_native.STAT_SLOTS * 2 * K, device="cuda", dtype=torch.float64)
    yA = C.conv_fwd(a, w, 1, 1, p, p, True, tile[0], tile[1], splits, sums=sA, stages=stages)[0]

    rmB, rvB = rm0.clone(), rv0.clone()
    xout = torch.empty_like(y0)
    stats = torch.empty(2, Cin, device="cuda")
    sB = torch.zeros_like(sA)
    yB = C.conv_fwd(y0, w, 1, 1, p, p, True, tile[0], tile[1], splits, sums=sB, stages=stages, xf_sums=sums, xf_w=g,
                    xf_b=b, xf_rm=rmB, xf_rv=rvB, xf_momentum=0.1, xf_eps=1e-5, xf_out=xout, xf_stats=stats)[0]
    torch.cuda.synchronize()
    assert torch.equal(xout, a)
    assert torch.equal(stats[0], mean) and torch.equal(stats[1], invstd)
    assert torch.equal(rmA, rmB) and torch.equal(rvA, rvB)
    assert torch.equal(yA, yB)
    torch.testing.assert_close(sA, sB, rtol=1e-12, atol=1e-9)  # f64 atomics: arrival order may vary
    ref = torch.nn.functional.conv2d(a.float(), w.float(), padding=p)
    torch.testing.assert_close(yB.float(), ref, rtol=2e-2, atol=2e-2)


def test_conv_xf_refuses_uncovered_geometry():
    """The side output needs the centre tap to cover every input pixel: stride 2 is refused."""
    from hyperion.ops import _native

    C = _native.native()
    y0 = torch.randn(2, 64, 8, 8, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 3, 3, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    sums = _sums_of(y0, _native.STAT_SLOTS)
    with pytest.raises(RuntimeError):
        C.conv_fwd(y0, w, 2, 2, 1, 1, True, xf_sums=sums, xf_out=torch.empty_like(y0),
                   xf_stats=torch.empty(2, 64, device="cuda"))


def _resnet_step(fuse: bool, monkeypatch):
    from hyperion.models.resnet import resnet50
    from hyperion.ops import _native
    from hyperion.ops import conv as conv_mod
    from hyperion.train.amp import cast_for_compute

    monkeypatch.setattr(conv_mod, "FUSE_BN_APPLY", fuse)
    torch.manual_seed(0)
    m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x = torch.randn(4, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    _native.reset_counters()
    out = m(x)
    loss = out.float().square().mean()
    loss.backward()
    torch.cuda.synchronize()
    cnt = dict(_native.counters())
    grads = {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}
    bufs = {n: b.detach().clone() for n, b in m.named_buffers()}
    return float(loss), out.detach().float(), grads, bufs, cnt


@pytest.mark.parametrize("only_1x1", [False, True])
def test_resnet50_step_with_fused_bn_apply_matches_unfused(monkeypatch, only_1x1):
    from hyperion.ops import conv as conv_mod

    monkeypatch.setattr(conv_mod, "XF_ONLY_1X1", only_1x1)
    # the plain conv's plans for the fused consumers too: identical accumulation order, so the
    # comparison is exact up to atomics order (a different tile changes bf16 roundings, which a
    # batch-4 ResNet's 16-sample layer4 BatchNorms amplify)
    monkeypatch.setattr(conv_mod, "XF_TILE", None)
    l0, o0, g0, b0, c0 = _resnet_step(False, monkeypatch)
    l1, o1, g1, b1, c1 = _resnet_step(True, monkeypatch)
    # every bottleneck's bn2 (the 1x1 conv3 consumer), and bn1 where conv2 has stride 1: 16 + 13
    assert c1.get("conv_xf") == (16 if only_1x1 else 29) and not c1.get("bn_apply_materialized"), c1
    assert not c0.get("conv_xf")
    torch.testing.assert_close(o1, o0, rtol=1e-2, atol=1e-2)
    assert abs(l1 - l0) <= 1e-3 * abs(l0)
    for n in g0:
        rel = float((g1[n] - g0[n]).norm() / (g0[n].norm() + 1e-12))
        assert rel < 2e-2, (n, rel)
    for n in b0:
        torch.testing.assert_close(b1[n].float(), b0[n].float(), rtol=1e-3, atol=1e-4)


def test_deferred_bn_materialized_for_a_non_fusable_consumer(monkeypatch):
    """A deferred conv -> BN -> ReLU output reaching a consumer that cannot apply it (a stride-2
    conv) is materialized by the standalone apply pass first — same forward and gradients."""
    from hyperion.ops import _native
    from hyperion.ops import conv as conv_mod

    monkeypatch.setattr(conv_mod, "FUSE_BN_APPLY", True)
    from hyperion.ops.batchnorm import BatchNormAct2d
    from hyperion.ops.conv import conv_bn_act

    torch.manual_seed(0)
    c1 = torch.nn.Conv2d(64, 64, 1, bias=False).cuda().bfloat16().to(memory_format=torch.channels_last)
    c2 = torch.nn.Conv2d(64, 128, 3, stride=2, padding=1, bias=False).cuda().bfloat16().to(
        memory_format=torch.channels_last)
    b1, b2 = BatchNormAct2d(64, act=True).cuda(), BatchNormAct2d(128, act=True).cuda()
    x0 = torch.randn(4, 64, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    res = []
    for defer in (False, True):
        for mod in (c1, c2, b1, b2):
            mod.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        _native.reset_counters()
        y = conv_bn_act(c2, b2, conv_bn_act(c1, b1, x, defer=defer))
        y.float().square().mean().backward()
        torch.cuda.synchronize()
        res.append((y.detach().clone(), x.grad.clone(), c1.weight.grad.clone(), b1.weight.grad.clone(),
                    dict(_native.counters())))
    assert res[1][4].get("bn_apply_materialized") == 1 and not res[1][4].get("conv_xf")
    for a, b in zip(res[0][:4], res[1][:4]):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-3)
