"""Local HF checkpoints for the Llama fine-tune (models/hf_checkpoint.py).

A random tiny Llama is written in the HF sharded safetensors layout (config.json, index, several
shards), reloaded bit-exactly through ``LlamaForCausalLM.from_pretrained`` (weights only, no
pickle), fine-tuned with LoRA on top, and picked up by ``train_llama_fsdp(model_id=<dir>)``.
Reference: ``02_development/distributed_utils.py:458, 465-468, 484-487`` (``from_pretrained``).
"""
import json
import os

import pytest
import torch


def _tiny(seed=0):
    from hyperion.models.llama import LlamaConfig, LlamaForCausalLM

    torch.manual_seed(seed)
    return LlamaForCausalLM(LlamaConfig.tiny(num_hidden_layers=2))


def test_sharded_roundtrip_bit_exact(tmp_path):
    from hyperion.models.hf_checkpoint import INDEX, is_hf_dir, iter_shard_names, save_hf_checkpoint
    from hyperion.models.llama import LlamaForCausalLM

    m = _tiny()
    files = save_hf_checkpoint(m, str(tmp_path), max_shard_bytes=200_000)
    assert len(files) >= 3 and is_hf_dir(str(tmp_path))
    idx = json.load(open(tmp_path / INDEX))
    assert set(idx["weight_map"]) == {k for k, _ in m.named_parameters()}
    assert list(iter_shard_names(str(tmp_path))) == sorted(files)
    cfg = json.load(open(tmp_path / "config.json"))
    assert cfg["hidden_size"] == m.config.hidden_size and cfg["model_type"] == "llama"
    r = LlamaForCausalLM.from_pretrained(str(tmp_path))
    assert r.config.num_hidden_layers == 2 and r.config.vocab_size == m.config.vocab_size
    for (k, a), (k2, b) in zip(m.state_dict().items(), r.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    # bf16 cast on load (the reference's torch_dtype=bfloat16)
    rb = LlamaForCausalLM.from_pretrained(str(tmp_path), torch_dtype=torch.bfloat16)
    assert rb.lm_head.weight.dtype == torch.bfloat16
    assert torch.equal(rb.lm_head.weight, m.lm_head.weight.to(torch.bfloat16))


def test_strict_and_safetensors_only(tmp_path):
    from safetensors.torch import save_file

    from hyperion.models.hf_checkpoint import load_hf_weights, save_hf_checkpoint

    m = _tiny()
    save_hf_checkpoint(m, str(tmp_path))  # one shard: model.safetensors
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd.pop("model.norm.weight")
    sd["model.layers.0.self_attn.rotary_emb.inv_freq"] = torch.ones(4)  # an HF buffer: skipped
    save_file(sd, str(tmp_path / "model.safetensors"))
    with pytest.raises(KeyError):
        load_hf_weights(_tiny(1), str(tmp_path))
    got = load_hf_weights(_tiny(1), str(tmp_path), strict=False)
    assert got["missing"] == ["model.norm.weight"] and got["skipped"]
    with open(tmp_path / "model.safetensors.index.json", "w") as f:
        json.dump({"weight_map": {"lm_head.weight": "pytorch_model.bin"}}, f)
    with pytest.raises(ValueError):
        load_hf_weights(_tiny(1), str(tmp_path))


def test_lora_finetune_on_loaded_weights(tmp_path):
    from hyperion.models.hf_checkpoint import save_hf_checkpoint
    from hyperion.models.llama import LlamaForCausalLM
    from hyperion.models.lora import apply_lora

    src = _tiny(3)
    save_hf_checkpoint(src, str(tmp_path), max_shard_bytes=300_000)
    m = apply_lora(LlamaForCausalLM.from_pretrained(str(tmp_path)), r=8, alpha=16, dropout=0.0)
    frozen = {k: v.clone() for k, v in m.named_parameters() if not v.requires_grad}
    assert frozen and torch.equal(frozen["lm_head.weight"], src.lm_head.weight)
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    ids = torch.randint(0, m.config.vocab_size, (2, 17))
    losses = []
    for _ in range(3):
        opt.zero_grad()
        loss = m(ids, labels=ids).loss
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
    assert losses[-1] < losses[0]
    for k, v in m.named_parameters():
        if not v.requires_grad:
            assert torch.equal(v, frozen[k]), k  # the base stays the checkpoint's


def test_trainer_loads_local_model_id(tmp_path):
    from hyperion.models.hf_checkpoint import save_hf_checkpoint
    from hyperion.train.distributed import RunOptions, train_llama_fsdp

    ck = tmp_path / "llama_ckpt"
    save_hf_checkpoint(_tiny(5), str(ck), max_shard_bytes=250_000)
    opts = RunOptions(synthetic=True, seed=1, save=False, dataset_size=4, max_steps_per_epoch=2, log=lambda s: None)
    r = train_llama_fsdp(0, 1, epochs=1, base_dir=str(tmp_path), model_id=str(ck), lora=True, batch_size=2,
                         progress_every=0, opts=opts)
    assert r["weights"] == f"pretrained:{ck}"
    assert r["history"] and torch.isfinite(torch.tensor(r["history"][0]["loss"]))
    r2 = train_llama_fsdp(0, 1, epochs=1, base_dir=str(tmp_path), model_id="no/such-hub-id", lora=True,
                          batch_size=2, progress_every=0, opts=opts,
                          config=__import__("hyperion.models.llama", fromlist=["LlamaConfig"]).LlamaConfig.tiny())
    assert r2["weights"] == "random-init"


def test_tied_embeddings_share_one_parameter(tmp_path):
    """tie_word_embeddings: the LM head IS the embedding Parameter after loading (a copy
    drifted apart during training); only one tensor is saved."""
    from hyperion.models.hf_checkpoint import save_hf_checkpoint
    from hyperion.models.llama import LlamaConfig, LlamaForCausalLM

    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig.tiny(num_hidden_layers=1, tie_word_embeddings=True))
    assert m.lm_head.weight is m.model.embed_tokens.weight
    save_hf_checkpoint(m, str(tmp_path))
    r = LlamaForCausalLM.from_pretrained(str(tmp_path))
    assert r.lm_head.weight is r.model.embed_tokens.weight
    assert torch.equal(r.lm_head.weight, m.lm_head.weight)
    opt = torch.optim.SGD(r.parameters(), lr=0.1)
    ids = torch.randint(0, 512, (2, 9))
    r(ids, labels=ids).loss.backward()
    opt.step()
    assert r.lm_head.weight is r.model.embed_tokens.weight  # still one tensor after a step


@pytest.mark.parametrize("field,value", [("rope_scaling", {"rope_type": "llama3", "factor": 8.0}),
                                         ("attention_bias", True), ("head_dim", 48), ("hidden_act", "gelu")])
def test_unsupported_config_fields_refused(tmp_path, field, value):
    from hyperion.models.hf_checkpoint import load_llama_config, save_hf_checkpoint

    save_hf_checkpoint(_tiny(), str(tmp_path))
    cfg = json.load(open(tmp_path / "config.json"))
    cfg[field] = value
    json.dump(cfg, open(tmp_path / "config.json", "w"))
    with pytest.raises(ValueError, match=field):
        load_llama_config(str(tmp_path))
