"""``_native.apply_fn``: autograd Functions run through ``apply`` with grad mode on, and as a bare
forward on a stand-in ctx under ``no_grad`` (inference without autograd-node host overhead)."""
import torch


class _Scale(torch.autograd.Function):
    calls = []

    @staticmethod
    def forward(ctx, x, s):
        _Scale.calls.append(type(ctx).__name__)
        ctx.save_for_backward(x if ctx.needs_input_grad[0] else None)
        ctx.s = s
        return x * s

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


def test_apply_fn_grad_and_no_grad():
    from hyperion.ops._native import apply_fn

    x = torch.randn(5, requires_grad=True)
    y = apply_fn(_Scale, x, 3.0)
    assert y.grad_fn is not None
    y.sum().backward()
    torch.testing.assert_close(x.grad, torch.full((5,), 3.0))
    with torch.no_grad():
        z = apply_fn(_Scale, x, 2.0)
    assert z.grad_fn is None and not z.requires_grad
    torch.testing.assert_close(z, x.detach() * 2.0)
    assert _Scale.calls[-1] == "_InferCtx" and _Scale.calls[-2] != "_InferCtx"
