"""Persistent conv launches (csrc/kernels/conv_persist.h): grid = the resident capacity, each
workgroup loops over tiles and issues the next tile's first loads behind the current epilogue.

Every variant the persistent path serves must give the plain launch's output BITWISE (same tile,
same K order, same epilogue) and BN statistics / column sums to the fp64 atomics' noise:

* forward + BN statistics (64x64, 128x64, 128x128 tiles; 1x1 and 3x3, stride 1 and 2);
* plain data gradient, stride 1 and the stride-2 phase split;
* data gradient with the BN-backward epilogue, LEAN (mode 1) and full (mode 2 + addend).

Reference: MIOpen fwd / bwd-data solvers (SURVEY §2.4 conv row) — launched per tile there.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

FWD = [  # (N, C, H, K, R, stride, pad, bm, bn)
    (8, 64, 56, 256, 1, 1, 0, 128, 128),
    (8, 64, 56, 64, 3, 1, 1, 128, 64),
    (4, 256, 14, 256, 3, 1, 1, 64, 64),
    (4, 128, 28, 128, 3, 2, 1, 64, 64),
    (3, 64, 17, 72, 1, 1, 0, 64, 64),  # ragged M and K
]


def _t(shape, g, scale=1.0):
    return (torch.randn(*shape, device="cuda", generator=g) * scale).bfloat16().contiguous(
        memory_format=torch.channels_last)


def _both(fn):
    from hyperion.ops import _native

    C_ = _native.native()
    try:
        C_.conv_set_persist(0)
        a = fn(C_)
        C_.conv_set_persist(1)
        b = fn(C_)
        torch.cuda.synchronize()
    finally:
        C_.conv_set_persist(0)
    return a, b


def _close_sums(a, b):
    torch.testing.assert_close(b, a, rtol=1e-9, atol=1e-9 * a.abs().max().item() + 1e-12)


@pytest.mark.parametrize("shape", FWD)
def test_persist_forward_stats(shape):
    from hyperion.ops import _native

    N, C, H, K, R, s, p, bm, bn = shape
    g = torch.Generator(device="cuda").manual_seed(0)
    x = _t((N, C, H, H), g)
    w = _t((K, C, R, R), g, 0.05)
    slots = _native.STAT_SLOTS

    def run(C_):
        sums = torch.zeros(slots * 2 * K, device="cuda", dtype=torch.float64)
        y = C_.conv_fwd(x, w, s, s, p, p, True, bm=bm, bn=bn, splits=1, sums=sums)[0]
        return y, sums.view(slots, 2, K).sum(0)

    (y0, s0), (y1, s1) = _both(run)
    assert torch.equal(y1, y0)
    _close_sums(s0, s1)
    y32 = torch.nn.functional.conv2d(x.float(), w.float(), stride=s, padding=p)
    assert ((y0.float() - y32).norm() / y32.norm()).item() < 1e-2


DGRAD = [  # (N, C, H, K, R, stride, pad): the conv's input [N, C, H, H], filter [K, C, R, R]
    (8, 64, 56, 256, 1, 1, 0),
    (4, 64, 28, 64, 3, 1, 1),
    (4, 128, 28, 128, 3, 2, 1),
]


def _dgrad_kw(shape):
    N, C, H, K, R, s, p = shape
    if s == 2 and R > 1:
        return dict(ph=p, pw=p, stride=2, H=H, W=H)
    return dict(ph=p, pw=p)


@pytest.mark.parametrize("shape", DGRAD)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_persist_dgrad(shape, mode):
    """mode 0: plain dX; 1: LEAN BN-backward epilogue; 2: full epilogue + addend."""
    from hyperion.ops import _native

    N, C, H, K, R, s, p = shape
    P = (H + 2 * p - R) // s + 1
    g = torch.Generator(device="cuda").manual_seed(1)
    w = _t((K, C, R, R), g, 0.05)
    dy = _t((N, K, P, P), g)
    kw = _dgrad_kw(shape)
    ph, pw = kw.pop("ph"), kw.pop("pw")
    yc = _t((N, C, H, H), g)
    bw = torch.rand(C, device="cuda", generator=g) + 0.5
    bb = torch.randn(C, device="cuda", generator=g) * 0.1
    mean = torch.randn(C, device="cuda", generator=g) * 0.1
    invstd = torch.rand(C, device="cuda", generator=g) + 0.5
    xout = torch.relu(yc.float() * (bw * invstd).view(1, -1, 1, 1) + (bb - mean * bw * invstd).view(1, -1, 1, 1))
    xout = xout.bfloat16().contiguous(memory_format=torch.channels_last)
    add = _t((N, C, H, H), g) if mode == 2 else None
    slots = _native.STAT_SLOTS

    def run(C_):
        if mode == 0:
            return C_.conv_dgrad(dy, w, ph, pw, bm=64, bn=64, **kw), None
        sums = torch.zeros(slots * 2 * C, device="cuda", dtype=torch.float64)
        dz = C_.conv_dgrad(dy, w, ph, pw, bm=64, bn=64, addend=add, bn_x=yc, bn_y=xout if mode == 2 else None,
                           bn_w=bw, bn_b=bb, bn_mean=mean, bn_invstd=invstd, bn_mode=mode, bn_sums=sums, **kw)
        return dz, sums.view(slots, 2, C).sum(0)

    (d0, s0), (d1, s1) = _both(run)
    assert torch.equal(d1, d0)
    if mode:
        _close_sums(s0, s1)


def test_persist_resnet50_step_matches_plain():
    """A ResNet-50 forward + backward with persistent forward / data-gradient convs: loss and
    gradients equal the plain launches' to the BN statistics atomics' noise."""
    from hyperion.models.resnet import resnet50
    from hyperion.ops import _native
    from hyperion.train.amp import cast_for_compute

    torch.manual_seed(0)
    m = resnet50(num_classes=16).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x0 = torch.randn(8, 3, 96, 96, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    gy = torch.randn(8, 16, device="cuda").bfloat16()
    C_ = _native.native()

    def run(on):
        C_.conv_set_persist(on)
        try:
            for q in m.parameters():
                q.grad = None
            out = m(x0)
            out.backward(gy)
            torch.cuda.synchronize()
            return out.float().clone(), [q.grad.float().clone() for q in m.parameters()]
        finally:
            C_.conv_set_persist(0)

    (o0, ref), (o0b, ref2), (o1, got) = run(0), run(0), run(1)
    onoise = (o0b - o0).norm().item()
    assert (o1 - o0).norm().item() <= 4 * onoise + 1e-2 * o0.norm().item()
    for u, u2, v in zip(ref, ref2, got):
        noise = (u2 - u).norm().item()
        assert (v - u).norm().item() <= 4 * noise + 1e-2 * u.norm().item() + 1e-6
