"""LoRA: PEFT layout/keys, fused autograd == reference composition, adapter save/load, merge."""
import json

import torch

from hyperion.models.llama import LlamaConfig, LlamaForCausalLM
from hyperion.models.lora import LoRALinear, apply_lora, load_adapter, merge_lora, save_adapter, trainable_parameters
from hyperion.ops.lora import lora_linear, lora_linear_reference


def test_lora_linear_matches_reference_grads():
    torch.manual_seed(0)
    x = torch.randn(3, 5, 32, requires_grad=True)
    w, b = torch.randn(24, 32), torch.randn(24)
    a = torch.randn(4, 32, requires_grad=True)
    bm = torch.randn(24, 4, requires_grad=True)
    y = lora_linear(x, w, b, a, bm, 2.0, 0.0)
    xr, ar, br = (t.detach().clone().requires_grad_(True) for t in (x, a, bm))
    yr = lora_linear_reference(xr, w, b, ar, br, 2.0)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for u, v in ((x, xr), (a, ar), (bm, br)):
        torch.testing.assert_close(u.grad, v.grad, rtol=1e-4, atol=1e-5)


def test_lora_dropout_mask_regenerated_consistently():
    torch.manual_seed(0)
    x = torch.randn(64, 32, requires_grad=True)
    w = torch.randn(16, 32)
    a = torch.randn(4, 32, requires_grad=True)
    bm = torch.randn(16, 4, requires_grad=True)
    y = lora_linear(x, w, None, a, bm, 1.0, 0.5)
    # recover the mask the forward used: y - base = ((x*m) A^T) B^T; check grads with finite differences
    # of a linear function: d/dB of sum(y * g) = g^T t
    g = torch.randn_like(y)
    y.backward(g)
    base = x.detach() @ w.t()
    t = torch.linalg.lstsq(bm.detach(), (y.detach() - base).t()).solution.t()  # [N, r] = drop(x) A^T
    torch.testing.assert_close(bm.grad, g.t() @ t, rtol=1e-3, atol=1e-3)


def test_apply_lora_llama_keys_and_trainable_count():
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    m = apply_lora(LlamaForCausalLM(cfg), r=16, alpha=32, dropout=0.05)
    keys = set(m.state_dict())
    assert "model.layers.0.self_attn.q_proj.base_layer.weight" in keys
    assert "model.layers.0.self_attn.q_proj.lora_A.default.weight" in keys
    assert "model.layers.1.self_attn.o_proj.lora_B.default.weight" in keys
    h = cfg.hidden_size
    assert trainable_parameters(m) == cfg.num_hidden_layers * 4 * (16 * h + h * 16)
    # Llama-2-7B: 16,777,216 trainable
    assert 32 * 4 * (16 * 4096 * 2) == 16_777_216


def test_lora_zero_init_is_identity_and_trains():
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    base = LlamaForCausalLM(cfg).eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 12))
    ref = base(ids).logits.detach()
    m = apply_lora(base).eval()
    torch.testing.assert_close(m(ids).logits, ref)
    m.train()
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    l0 = None
    for _ in range(5):
        loss = m(ids, labels=ids).loss
        l0 = l0 if l0 is not None else loss.item()
        loss.backward()
        opt.step()
        opt.zero_grad()
    assert loss.item() < l0
    assert all(p.grad is None for n, p in m.named_parameters() if "base_layer" in n)


def test_adapter_save_load_roundtrip_and_merge(tmp_path):
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    m = apply_lora(LlamaForCausalLM(cfg))
    for mod in m.modules():
        if isinstance(mod, LoRALinear):
            torch.nn.init.normal_(mod.lora_B["default"].weight, std=0.1)
    save_adapter(m, str(tmp_path / "adapter"))
    conf = json.loads((tmp_path / "adapter" / "adapter_config.json").read_text())
    assert conf["r"] == 16 and conf["lora_alpha"] == 32 and conf["peft_type"] == "LORA"
    from safetensors.torch import load_file

    keys = set(load_file(str(tmp_path / "adapter" / "adapter_model.safetensors")))
    assert "base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight" in keys
    torch.manual_seed(1)
    m2 = apply_lora(LlamaForCausalLM(cfg))
    m2.load_state_dict({k: v for k, v in m.state_dict().items() if "lora" not in k}, strict=False)
    load_adapter(m2, str(tmp_path / "adapter"))
    ids = torch.randint(0, cfg.vocab_size, (1, 8))
    m.eval(), m2.eval()
    torch.testing.assert_close(m(ids).logits, m2(ids).logits)
    merged = merge_lora(m2)
    torch.testing.assert_close(merged(ids).logits, m(ids).logits, rtol=1e-4, atol=1e-4)


def test_lora_linear_dropout_grads_match_reference():
    """Dropout path: same draws (seeded), reference = base + s * ((x * keep / (1-p)) A^T) B^T."""
    from hyperion.ops.lora import lora_linear, lora_linear_reference

    torch.manual_seed(1)
    x = torch.randn(2, 5, 32, dtype=torch.float64, requires_grad=True)
    w = torch.randn(24, 32, dtype=torch.float64)
    a = torch.randn(4, 32, dtype=torch.float64, requires_grad=True)
    b = torch.randn(24, 4, dtype=torch.float64, requires_grad=True)
    p, s = 0.3, 2.0
    torch.manual_seed(7)
    y = lora_linear(x, w, None, a, b, s, p)
    torch.manual_seed(7)
    keep = torch.empty(10, 32, dtype=torch.float64).bernoulli_(1 - p).view(2, 5, 32)
    xr, ar, br = (t.detach().clone().requires_grad_(True) for t in (x, a, b))
    yr = lora_linear_reference(xr, w, None, ar, br, s, mask=keep / (1 - p))
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for u, v in ((y, yr), (x.grad, xr.grad), (a.grad, ar.grad), (b.grad, br.grad)):
        torch.testing.assert_close(u, v)
