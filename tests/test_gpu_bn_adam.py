"""GPU numerics: fused BN(+res)(+ReLU) and multi-tensor Adam vs PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_bn(x, res, w, b, rm, rv, training, mom, eps, act):
    y = F.batch_norm(x, rm, rv, w, b, training, mom, eps)
    if res is not None:
        y = y + res
    return F.relu(y) if act else y


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [64, 256, 2048])
@pytest.mark.parametrize("act,use_res", [(True, False), (True, True), (False, False)])
def test_bn_act_matches_reference(dtype, C, act, use_res):
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import _BNActFn

    assert _native.available(), "native extension must load on the GPU box"
    torch.manual_seed(0)
    N, H, W = 4, 7, 5
    dev = "cuda"
    x = (torch.randn(N, C, H, W, device=dev) * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x) if use_res else None
    w = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()

    xr = x.detach().float().requires_grad_(True)
    resr = res.detach().float().requires_grad_(True) if use_res else None
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = _ref_bn(xr, resr, wr, br, rm2, rv2, True, 0.1, 1e-5, act)

    xn = x.detach().requires_grad_(True)
    resn = res.detach().requires_grad_(True) if use_res else None
    wn = w.clone().requires_grad_(True)
    bn = b.clone().requires_grad_(True)
    yn = _BNActFn.apply(xn, resn, wn, bn, rm, rv, 0.1, 1e-5, True, act)

    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(yn.float(), yr, atol=tol, rtol=tol)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(rv, rv2, atol=1e-4, rtol=1e-3)

    gy = torch.randn_like(yr)
    yr.backward(gy)
    yn.backward(gy.to(dtype).contiguous(memory_format=torch.channels_last))
    gtol = 2e-4 if dtype == torch.float32 else 6e-2
    torch.testing.assert_close(xn.grad.float(), xr.grad, atol=gtol, rtol=gtol)
    torch.testing.assert_close(wn.grad, wr.grad, atol=gtol * C, rtol=gtol)
    torch.testing.assert_close(bn.grad, br.grad, atol=gtol * C, rtol=gtol)
    if use_res:
        torch.testing.assert_close(resn.grad.float(), resr.grad, atol=gtol, rtol=gtol)


def test_bn_eval_mode():
    from hyperion.ops.batchnorm import BatchNormAct2d

    torch.manual_seed(1)
    m = BatchNormAct2d(128, act=True).cuda()
    m.running_mean.uniform_(-1, 1)
    m.running_var.uniform_(0.5, 2)
    m.eval()
    x = torch.randn(2, 128, 6, 6, device="cuda").contiguous(memory_format=torch.channels_last)
    y = m(x)
    yr = F.relu(F.batch_norm(x, m.running_mean, m.running_var, m.weight, m.bias, False, 0.1, 1e-5))
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-5)


def test_fused_adam_matches_torch():
    from hyperion.ops import FusedAdam

    torch.manual_seed(0)
    shapes = [(64, 3, 7, 7), (1000, 2048), (1000,), (3,), (8191,)]
    ps = [torch.randn(s, device="cuda", requires_grad=True) for s in shapes]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    for adamw, wd in [(False, 0.0), (False, 1e-2), (True, 1e-2)]:
        opt = FusedAdam(ps, lr=1e-3, weight_decay=wd, adamw=adamw)
        ref = (torch.optim.AdamW if adamw else torch.optim.Adam)(qs, lr=1e-3, weight_decay=wd)
        for _ in range(5):
            for p, q in zip(ps, qs):
                g = torch.randn_like(p)
                p.grad = g.clone()
                q.grad = g.clone()
            opt.step()
            ref.step()
        for p, q in zip(ps, qs):
            torch.testing.assert_close(p, q, atol=1e-5, rtol=1e-4)


def test_stream_kernels():
    from hyperion.ops import _native

    C = _native.native()
    n = 1 << 20
    a = torch.randn(n, device="cuda")
    b = torch.randn(n, device="cuda")
    c = torch.empty_like(a)
    C.stream(2, a, b, c, 0.0, False, 0)
    torch.testing.assert_close(c, a + b)
    C.stream(3, a, b, c, 3.0, True, 0)
    torch.testing.assert_close(c, a + 3.0 * b)
    C.stream(0, a, None, c, 0.0, False, 0)
    torch.testing.assert_close(c, a)


def test_resnet50_native_step_runs_and_matches_torch_path():
    """One bf16 training step through the fused kernels vs the torch path on identical weights."""
    import copy
    import os

    from hyperion.models import resnet50

    torch.manual_seed(0)
    m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    m2 = copy.deepcopy(m)
    x = torch.randn(8, 3, 96, 96, device="cuda").contiguous(memory_format=torch.channels_last)
    out = m(x)  # fp32 end to end: fused BN kernels vs torch BN/add/relu
    out.sum().backward()
    os.environ["HYPERION_KERNELS"] = "torch"
    try:
        out2 = m2(x)
        out2.sum().backward()
    finally:
        os.environ.pop("HYPERION_KERNELS", None)
    torch.testing.assert_close(out, out2, atol=2e-3, rtol=2e-3)
    for (n1, p1), (_, p2) in zip(m.named_parameters(), m2.named_parameters()):
        cos = F.cosine_similarity(p1.grad.flatten().double(), p2.grad.flatten().double(), dim=0)
        assert cos > 0.999, (n1, float(cos))
    for (n1, b1), (_, b2) in zip(m.named_buffers(), m2.named_buffers()):
        if b1.is_floating_point():
            torch.testing.assert_close(b1, b2, atol=1e-4, rtol=1e-3)


def test_fused_adam_master_weights_bf16():
    """bf16 compute copies + fp32 masters: master tracks fp32 Adam exactly; copy = rounded master."""
    from hyperion.ops import FusedAdam

    torch.manual_seed(0)
    shapes = [(256, 64, 1, 1), (1000, 2048), (1000,)]
    ref = [torch.randn(s, device="cuda").bfloat16().float().requires_grad_(True) for s in shapes]
    lowp = [r.detach().bfloat16().requires_grad_(True) for r in ref]
    opt = FusedAdam(lowp, lr=1e-3)
    ropt = torch.optim.Adam(ref, lr=1e-3)
    for _ in range(4):
        for p, r in zip(lowp, ref):
            g = torch.randn_like(r)
            p.grad = g.bfloat16()
            r.grad = g.bfloat16().float()
        opt.step()
        ropt.step()
    for p, r in zip(lowp, ref):
        torch.testing.assert_close(opt.state[p]["master"], r.detach(), atol=1e-5, rtol=1e-4)
        # the compute copy is exactly the rounded master (the master itself may differ from the
        # torch fp32 trajectory by an ulp, which can flip a bf16 rounding: compare to the master)
        torch.testing.assert_close(p.detach(), opt.state[p]["master"].bfloat16(), atol=0, rtol=0)


def test_fused_adam_channels_last_params_take_native_path():
    from hyperion.models import resnet18
    from hyperion.ops import FusedAdam

    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = FusedAdam(m.parameters())
    x = torch.randn(2, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    m(x).sum().backward()
    opt.step()
    assert opt._tables._tables, "channels-last params must use the multi-tensor kernel"


def test_fused_adam_zero_grad_in_step():
    from hyperion.ops.optim import FusedAdam

    torch.manual_seed(0)
    ps = [torch.randn(1000, device="cuda", requires_grad=True), torch.randn(33, 7, device="cuda", requires_grad=True)]
    ref = [p.detach().clone().requires_grad_(True) for p in ps]
    o1 = FusedAdam(ps, lr=1e-2, zero_grad_in_step=True)
    o2 = torch.optim.Adam(ref, lr=1e-2)
    for _ in range(3):
        for p, r in zip(ps, ref):
            g = torch.randn_like(p)
            p.grad = g.clone() if p.grad is None else p.grad.add_(g)  # accumulate into the zeroed grad
            r.grad = g.clone()
        o1.step()
        o2.step()
        for p in ps:
            assert torch.count_nonzero(p.grad) == 0
        o1.zero_grad(set_to_none=False)  # no-op: already zero
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p, r, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("C", [64, 256, 4096, 6144])
def test_bn_combine_multichunk_matches_and_is_deterministic(C):
    """Large M / wide C: statistics summed by float atomics across many row blocks and finalized
    inline.  Atomic arrival order varies, so run-to-run results may differ in the last bits only
    (one bf16 ulp of an output at most), and all of them match the fp32 reference."""
    from hyperion.ops.batchnorm import _BNActFn

    torch.manual_seed(1)
    N, H, W = (32, 28, 28) if C <= 256 else (8, 8, 8)
    x = (torch.randn(N, C, H, W, device="cuda") * 1.5 + 0.25).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    gy = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)

    def run():
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        xn = x.detach().requires_grad_(True)
        wn, bn = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        yn = _BNActFn.apply(xn, None, wn, bn, rm, rv, 0.1, 1e-5, True, True)
        yn.backward(gy)
        return yn, xn.grad, wn.grad, bn.grad, rm, rv

    outs = [run() for _ in range(3)]
    for o in outs[1:]:
        for a, b2 in zip(outs[0], o):
            assert torch.equal(a, b2), "fp64 statistics sums: reproducible"
    xr = x.detach().float().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rm2, rv2 = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    yr = _ref_bn(xr, None, wr, br, rm2, rv2, True, 0.1, 1e-5, True)
    yr.backward(gy.float())
    yn, gx, gw, gb, rm, rv = outs[0]
    torch.testing.assert_close(yn.float(), yr, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(rv, rv2, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(gx.float(), xr.grad, atol=6e-2, rtol=6e-2)
    M = N * H * W
    torch.testing.assert_close(gw, wr.grad, atol=1e-3 * M ** 0.5, rtol=2e-2)
    torch.testing.assert_close(gb, br.grad, atol=1e-3 * M ** 0.5, rtol=2e-2)


@pytest.mark.parametrize("shape", [(32, 512, 7, 7), (32, 2048, 7, 7), (32, 256, 14, 14), (32, 1024, 14, 14),
                                   (3, 64, 5, 5)])
@pytest.mark.parametrize("act,use_res", [(True, False), (True, True), (False, False)])
def test_bn_small_m_paths_match_general_path(shape, act, use_res):
    """Small-M fast paths (finalize folded into the apply; one-launch backward) vs the general
    3-kernel paths and the fp32 reference, through the conv-partials entry (ResNet layer3/4)."""
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import _BNActFn

    C_ = _native.native()
    N, C, H, W = shape
    torch.manual_seed(2)
    x = (torch.randn(N, C, H, W, device="cuda") * 1.3 + 0.2).bfloat16().contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x) if use_res else None
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    gy = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)

    def run(small):
        C_.bn_set_small_paths(small)
        try:
            rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
            xn = x.detach().requires_grad_(True)
            rn = res.detach().requires_grad_(True) if use_res else None
            wn, bn = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
            yn = _BNActFn.apply(xn, rn, wn, bn, rm, rv, 0.1, 1e-5, True, act)
            yn.backward(gy)
            return [yn, xn.grad, wn.grad, bn.grad, rm, rv] + ([rn.grad] if use_res else [])
        finally:
            C_.bn_set_small_paths(True)

    fast, slow = run(True), run(False)
    M = N * H * W
    for i, (a, c) in enumerate(zip(fast, slow)):
        tol = 1e-3 * M ** 0.5 if i in (2, 3) else 2e-2
        torch.testing.assert_close(a.float(), c.float(), atol=tol, rtol=2e-2, msg=f"output {i}")
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True) if use_res else None
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = _ref_bn(xr, rr, wr, br, torch.zeros(C, device="cuda"), torch.ones(C, device="cuda"), True, 0.1, 1e-5, act)
    yr.backward(gy.float())
    torch.testing.assert_close(fast[0].float(), yr, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(fast[1].float(), xr.grad, atol=6e-2, rtol=6e-2)


@pytest.mark.parametrize("shape", [(32, 64, 56, 56), (32, 256, 56, 56), (8, 128, 28, 28), (4, 2048, 7, 7)])
@pytest.mark.parametrize("act,use_res", [(True, False), (True, True)])
def test_bn_atomic_sums_arena_and_retain_graph(shape, act, use_res):
    """Statistics as atomic per-channel sums finalized inline by the consumers, with the
    accumulators taken from one pre-zeroed arena (zero_scope, learnt size on the 2nd pass): matches
    the fp32 reference; a second backward over the same graph (retain_graph) takes fresh zeroed
    sums and reproduces the first backward's gradients."""
    from hyperion.ops import _native
    from hyperion.ops.batchnorm import _BNActFn

    N, C, H, W = shape
    torch.manual_seed(3)
    x = (torch.randn(N, C, H, W, device="cuda") * 1.1 - 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x) if use_res else None
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    gy = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)

    class Owner:
        pass

    owner = Owner()
    outs = []
    for it in range(2):  # 1st: learns the arena size (fresh zeros); 2nd: one arena slice per call
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        xn = x.detach().requires_grad_(True)
        rn = res.detach().requires_grad_(True) if use_res else None
        wn, bn = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        with _native.zero_scope(owner, "fwd", x.device):
            yn = _BNActFn.apply(xn, rn, wn, bn, rm, rv, 0.1, 1e-5, True, act)
        yn.backward(gy, retain_graph=True)
        first = [xn.grad.clone(), wn.grad.clone(), bn.grad.clone()]
        xn.grad = wn.grad = bn.grad = None
        yn.backward(gy)
        for a, c in zip(first, [xn.grad, wn.grad, bn.grad]):
            torch.testing.assert_close(a.float(), c.float(), atol=1e-2, rtol=1e-2)
        outs.append([yn, first[0], first[1], first[2], rm, rv])
    assert owner._zero_arena_sizes["fwd"] >= 4 * C
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True) if use_res else None
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rmr, rvr = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    yr = _ref_bn(xr, rr, wr, br, rmr, rvr, True, 0.1, 1e-5, act)
    yr.backward(gy.float())
    M = N * H * W
    for o in outs:
        torch.testing.assert_close(o[0].float(), yr, atol=3e-2, rtol=3e-2)
        torch.testing.assert_close(o[1].float(), xr.grad, atol=6e-2, rtol=6e-2)
        torch.testing.assert_close(o[2], wr.grad, atol=1e-3 * M ** 0.5, rtol=2e-2)
        torch.testing.assert_close(o[3], br.grad, atol=1e-3 * M ** 0.5, rtol=2e-2)
        torch.testing.assert_close(o[4], rmr, atol=1e-4, rtol=1e-3)
        torch.testing.assert_close(o[5], rvr, atol=1e-4, rtol=1e-3)
