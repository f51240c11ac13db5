"""Gradient links hold their source activation weakly (a strong ``link.src`` kept one
[B, S, E] activation per layer alive under non-reentrant activation checkpointing)."""
import gc

import torch


def test_residual_and_branch_links_do_not_own_their_source():
    from hyperion.ops.conv import BranchSumLink, ResidualLink

    x = torch.randn(4, 8)
    r, b = ResidualLink(x), BranchSumLink(x)
    assert r.src is x and b.src is x  # identity checks in the consumers still work
    y = torch.randn(4, 8)
    assert y is not r.src
    del x
    gc.collect()
    assert r.src is None and b.src is None  # the link did not keep the activation alive
    assert y is not r.src  # a dead link never matches a live tensor


def test_checkpointed_encoder_frees_link_sources():
    """Forward of a checkpointed encoder stack: once the layer inputs go out of scope, no link
    keeps them alive (the stored activations are exactly checkpointing's boundary tensors)."""
    from hyperion.models.transformer import encoder

    torch.manual_seed(0)
    enc = encoder(32, 4, 3, dim_feedforward=64, dropout=0.0, use_checkpoint=True).train()
    x = torch.randn(2, 5, 32, requires_grad=True)
    out = enc(x)
    out.sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    ref = encoder(32, 4, 3, dim_feedforward=64, dropout=0.0, use_checkpoint=False).train()
    ref.load_state_dict(enc.state_dict())
    x2 = x.detach().clone().requires_grad_(True)
    ref(x2).sum().backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-4, atol=1e-5)
