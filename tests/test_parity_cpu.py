"""The update-parity checks of tests/parity.py CAN fail (VERDICT r04 "next round" #5).

A reference schedule (4 Adam steps) against: an identical rerun (must pass), a run whose optimizer
skips one step, one that applies half an update once, and one that reuses a stale gradient — each
of the broken ones must fail the parameter-delta bound that the GPU graphed-vs-eager tests use
(2e-2), even though the skipped / halved ones pass the old absolute check (atol 2e-3 on the parameters).
"""
import pytest
import torch

from parity import assert_losses_match, snapshot, update_rel_err


def _run(mode: str, steps: int = 4):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 4))
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(1)
    data = [(torch.randn(8, 16, generator=g), torch.randn(8, 4, generator=g)) for _ in range(steps)]
    before = snapshot(m.named_parameters())
    losses, stale = [], None
    for i, (x, y) in enumerate(data):
        opt.zero_grad(set_to_none=False)
        loss = torch.nn.functional.mse_loss(m(x), y)
        loss.backward()
        losses.append(float(loss))
        if mode == "stale" and i == 1:
            stale = [p.grad.clone() for p in m.parameters()]
        if mode == "stale" and i == 2:
            for p, s in zip(m.parameters(), stale):
                p.grad.copy_(s)
        if mode == "skip" and i == 2:
            continue
        if mode == "half" and i == 2:
            for pg in opt.param_groups:
                pg["lr"] = 0.5e-3
        opt.step()
        for pg in opt.param_groups:
            pg["lr"] = 1e-3
    return before, snapshot(m.named_parameters()), losses


def test_identical_schedule_passes():
    b, ref, lr = _run("ok")
    b2, a, la = _run("ok")
    assert all(torch.equal(b[k], b2[k]) for k in b)
    assert update_rel_err(b, a, ref) == 0.0
    assert_losses_match(la, lr)


@pytest.mark.parametrize("mode", ["skip", "half", "stale"])
def test_broken_schedule_fails_delta_check(mode):
    b, ref, _ = _run("ok")
    _, bad, _ = _run(mode)
    if mode != "stale":  # the old check passes: every parameter is within atol=2e-3 of the reference ...
        for k in ref:
            torch.testing.assert_close(bad[k], ref[k], rtol=2e-2, atol=2e-3)
    # ... the delta check does not
    assert update_rel_err(b, bad, ref) > 2e-2


def test_broken_schedule_fails_loss_check():
    _, _, lr = _run("ok", steps=6)
    _, _, ls = _run("skip", steps=6)
    with pytest.raises(AssertionError):
        assert_losses_match(ls, lr, rtol=1e-6)
