"""CPU unit tests: model zoo shapes, parameter counts and reference-compatible state-dict keys."""
import torch
import torch.nn as nn

from hyperion.models.llama import LlamaConfig, LlamaForCausalLM, param_count
from hyperion.models.resnet import resnet18, resnet50
from hyperion.models.simple_lm import simple_lm_256, simple_lm_768
from hyperion.models.transformer import create_custom_transformer, count_params
from hyperion.models.vit import fallback_cnn, vit_b_16, vit_tiny


def test_param_counts_match_survey():
    # SURVEY §2.1 C14/C15/C5 and §2.5
    assert count_params(simple_lm_256()) == 28_411_985
    assert abs(count_params(simple_lm_768()) - 105.6e6) < 0.1e6
    assert count_params(create_custom_transformer()) == 18_914_304
    assert count_params(fallback_cnn()) == 212_328
    assert count_params(resnet18(num_classes=10)) == 11_181_642
    assert count_params(resnet50()) == 25_557_032
    assert count_params(vit_b_16()) == 86_567_656
    assert param_count(LlamaConfig.llama2_7b()) == 6_738_415_616


def test_simple_lm_keys_both_styles_and_torch_encoder_compat():
    m = simple_lm_256(vocab_size=100)
    keys = set(m.state_dict())
    assert {"embed.weight", "fc.weight", "fc.bias", "tr.layers.1.norm2.bias",
            "tr.layers.0.self_attn.in_proj_weight", "tr.layers.0.self_attn.out_proj.weight"} <= keys
    nb = simple_lm_256(vocab_size=100, key_style="notebook")
    assert "embedding.weight" in nb.state_dict() and "transformer.layers.0.linear1.weight" in nb.state_dict()
    # the encoder's keys equal nn.TransformerEncoder's, so a reference checkpoint loads
    ref = nn.TransformerEncoder(nn.TransformerEncoderLayer(256, 4), 2, enable_nested_tensor=False)
    ours = m.tr
    assert set(ref.state_dict()) == set(ours.state_dict())
    ours.load_state_dict(ref.state_dict())


def test_encoder_matches_torch_transformer_encoder_numerics():
    torch.manual_seed(0)
    ref = nn.TransformerEncoder(nn.TransformerEncoderLayer(64, 4, 128, dropout=0.0), 2, enable_nested_tensor=False)
    m = simple_lm_256(vocab_size=50, emb_dim=64, n_heads=4, ff_dim=128, dropout=0.0).tr
    m.load_state_dict(ref.state_dict())
    ref.eval(), m.eval()
    x = torch.randn(5, 3, 64)  # [S, B, E] for torch (batch_first=False)
    y_ref = ref(x)
    y = m(x.transpose(0, 1)).transpose(0, 1)
    torch.testing.assert_close(y, y_ref, rtol=1e-4, atol=1e-5)


def test_lm768_takes_seq_first_input():
    m = simple_lm_768(vocab_size=64)
    out = m(torch.randint(0, 64, (16, 2)))
    assert out.shape == (16, 2, 64)


def test_lm_forward_loss_equals_logits_ce():
    torch.manual_seed(0)
    m = simple_lm_256(vocab_size=97, dropout=0.0)
    ids = torch.randint(0, 97, (3, 12))
    ids[0, 8:] = 96
    x, y = ids[:, :-1], ids[:, 1:]
    l1 = m.forward_loss(x, y, ignore_index=96)
    l2 = nn.functional.cross_entropy(m(x).reshape(-1, 97), y.reshape(-1), ignore_index=96)
    torch.testing.assert_close(l1, l2, rtol=1e-5, atol=1e-6)
    g1 = torch.autograd.grad(l1, list(m.parameters()))
    g2 = torch.autograd.grad(l2, list(m.parameters()))
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def test_vit_keys_match_torchvision_layout():
    keys = set(vit_b_16().state_dict())
    for k in ("conv_proj.weight", "class_token", "encoder.pos_embedding", "encoder.ln.weight", "heads.head.weight",
              "encoder.layers.encoder_layer_11.mlp.3.bias", "encoder.layers.encoder_layer_0.self_attention.in_proj_weight",
              "encoder.layers.encoder_layer_0.ln_1.weight"):
        assert k in keys, k


def test_vit_checkpointing_same_grads():
    torch.manual_seed(0)
    m = vit_tiny()
    x = torch.randn(2, 3, 32, 32)
    nn.init.normal_(m.heads.head.weight, std=0.02)
    l1 = m(x).square().mean()
    g1 = torch.autograd.grad(l1, list(m.parameters()))
    m.use_checkpoint = True
    l2 = m(x).square().mean()
    g2 = torch.autograd.grad(l2, list(m.parameters()))
    torch.testing.assert_close(l1, l2)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b)


def test_llama_tiny_forward_backward_and_keys():
    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig.tiny())
    ids = torch.randint(0, 512, (2, 16))
    out = m(ids, labels=ids)
    out.loss.backward()
    assert torch.isfinite(out.loss)
    keys = set(m.state_dict())
    assert {"model.embed_tokens.weight", "lm_head.weight", "model.norm.weight",
            "model.layers.1.mlp.down_proj.weight", "model.layers.0.post_attention_layernorm.weight"} <= keys
    # loss equals HF semantics: shifted CE over logits
    logits = m(ids).logits
    ref = nn.functional.cross_entropy(logits[:, :-1].reshape(-1, 512), ids[:, 1:].reshape(-1))
    torch.testing.assert_close(out.loss, ref, rtol=1e-4, atol=1e-5)


def test_llama_padding_mask_and_causality():
    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig.tiny()).eval()
    ids = torch.randint(0, 512, (1, 10))
    full = m(ids).logits
    ids2 = ids.clone()
    ids2[0, 7:] = 3  # changing future tokens must not change earlier logits (causal)
    part = m(ids2).logits
    torch.testing.assert_close(full[:, :7], part[:, :7])


def test_resnet_cifar_one_step_cpu():
    # BASELINE.json config #1: ResNet-18 on a CIFAR-10-shaped synthetic batch, 1 step on CPU
    torch.manual_seed(0)
    m = resnet18(num_classes=10)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    x, y = torch.randn(4, 3, 32, 32), torch.randint(0, 10, (4,))
    loss = nn.functional.cross_entropy(m(x), y)
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)
