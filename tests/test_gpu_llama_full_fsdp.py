"""Llama full fine-tune under Hyperion FSDP (``train_llama_fsdp(lora=False)``: every weight
trainable, one unit per decoder layer, bf16 mixed precision) against the same model trained in
fp32 by plain torch ops and ``torch.optim.AdamW``.

Reference workload: ``02_development/distributed_utils.py:477-500, 540-550`` (torch FSDP,
``LlamaDecoderLayer`` wrap policy, bf16 ``MixedPrecision``).  Checks on a tiny config, one GPU:
the first step's loss and every parameter's gradient (unflattened from the FSDP shard) match the
fp32 reference, and over a few AdamW steps both losses fall together.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def test_llama_full_fsdp_matches_fp32_torch(monkeypatch):
    from hyperion.models.llama import LlamaConfig, LlamaDecoderLayer, LlamaForCausalLM
    from hyperion.ops.optim import FusedAdam
    from hyperion.parallel.fsdp import FSDP, MixedPrecision, transformer_auto_wrap_policy

    torch.manual_seed(0)
    cfg = LlamaConfig.tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=2, intermediate_size=512)
    base = LlamaForCausalLM(cfg).cuda()
    ref = copy.deepcopy(base)  # fp32, torch kernels
    names = {id(p): n for n, p in base.named_parameters()}
    bf = torch.bfloat16
    m = FSDP(base, auto_wrap_policy=transformer_auto_wrap_policy({LlamaDecoderLayer}),
             device_id=torch.device("cuda", 0), mixed_precision=MixedPrecision(bf, bf, bf))
    assert len(m.units) == cfg.num_hidden_layers + 1
    opt = FusedAdam(list(m.parameters()), lr=1e-3, weight_decay=0.01, adamw=True)
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.01)
    g = torch.Generator(device="cuda").manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), device="cuda", generator=g)

    losses, rlosses = [], []
    for step in range(4):
        opt.zero_grad(set_to_none=True)
        loss = m(ids, labels=ids).loss
        loss.backward()
        if step == 0:
            grads = {}
            for grp in m.flat_groups():
                if grp.flat_param.grad is None:
                    continue
                for p, o, n, shp in zip(grp.params, grp.offsets, grp.numels, grp.shapes):
                    grads[names[id(p)]] = grp.flat_param.grad[o:o + n].view(shp).clone()
        opt.step()
        losses.append(float(loss))

        monkeypatch.setenv("HYPERION_KERNELS", "torch")
        ropt.zero_grad(set_to_none=True)
        rloss = ref(ids, labels=ids).loss
        rloss.backward()
        if step == 0:
            assert set(grads) == {n for n, _ in ref.named_parameters()}
            for n, p in ref.named_parameters():
                assert _rel(grads[n], p.grad) < 0.06, n
        ropt.step()
        monkeypatch.delenv("HYPERION_KERNELS")
        rlosses.append(float(rloss))

    assert abs(losses[0] - rlosses[0]) <= 2e-2 * abs(rlosses[0])
    assert losses[-1] < losses[0] - 0.05 and rlosses[-1] < rlosses[0] - 0.05  # both train
    for a, b in zip(losses, rlosses):
        assert abs(a - b) <= 5e-2 * abs(b), (losses, rlosses)
