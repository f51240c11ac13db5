"""Local Hugging Face checkpoints for the Llama fine-tune: safetensors shards, weights only.

Reference: ``train_llama_fsdp`` starts from ``AutoModelForCausalLM.from_pretrained(model_id,
token=hf_token, torch_dtype=bfloat16)`` (``02_development/distributed_utils.py:458, 465-468,
484-487``).  There is no network on MI355X nodes here, so ``model_id`` is honoured as a
LOCAL directory in the HF layout:

* ``config.json`` — the HF ``LlamaConfig`` fields (vocab / hidden / intermediate sizes, layers,
  heads, kv heads, rope theta, rms eps, tied embeddings);
* ``model.safetensors`` or ``model.safetensors.index.json`` + ``model-0000k-of-0000n.safetensors``
  shards (``weight_map``: tensor name -> shard file).

Loading never unpickles: safetensors only (``.bin`` / ``.pt`` checkpoints are refused).  Tensors
are copied one by one into the parameters of an already-built :class:`LlamaForCausalLM` (HF key
names, so no renaming), converted to the parameter dtype on the way — peak host memory is one
tensor, not a state dict.  FSDP then flattens and shards the loaded parameters as usual, so every
rank starts its shard from the checkpoint.  HF-only buffers (``rotary_emb.inv_freq``) are skipped;
any other unexpected or missing key is an error (``strict=True``).

:func:`save_hf_checkpoint` writes the same layout (the CPU tests build a random model on disk and
reload it bit-exactly).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

INDEX = "model.safetensors.index.json"
SINGLE = "model.safetensors"
_SKIP_SUFFIXES = ("rotary_emb.inv_freq",)  # HF buffers recomputed by the model

_CFG_FIELDS = ("vocab_size", "hidden_size", "intermediate_size", "num_hidden_layers", "num_attention_heads",
               "num_key_value_heads", "max_position_embeddings", "rms_norm_eps", "rope_theta", "initializer_range",
               "pad_token_id", "tie_word_embeddings")


def is_hf_dir(path: Optional[str]) -> bool:
    """A local HF checkpoint directory (config + safetensors weights)?"""
    return (bool(path) and os.path.isdir(path) and os.path.isfile(os.path.join(path, "config.json"))
            and (os.path.isfile(os.path.join(path, INDEX)) or os.path.isfile(os.path.join(path, SINGLE))))


# config fields whose non-default values this Llama does not implement: refusing them beats a model
# that loads without error and runs with the wrong RoPE / projections (Llama-3.x rope_scaling, ...)
_UNSUPPORTED = {"rope_scaling": None, "attention_bias": False, "mlp_bias": False, "hidden_act": "silu",
                "pretraining_tp": 1}


def load_llama_config(path: str):
    from .llama import LlamaConfig

    with open(os.path.join(path, "config.json")) as f:
        raw = json.load(f)
    bad = {k: raw[k] for k, ok in _UNSUPPORTED.items() if k in raw and raw[k] is not None and raw[k] != ok}
    hd = raw.get("head_dim")
    if hd is not None and "hidden_size" in raw and "num_attention_heads" in raw and \
            hd != raw["hidden_size"] // raw["num_attention_heads"]:
        bad["head_dim"] = hd
    if bad:
        raise ValueError(f"{path}/config.json: unsupported Llama settings {bad} (this model implements plain "
                         f"RoPE, bias-free projections, SiLU, head_dim = hidden_size / heads)")
    kw = {k: raw[k] for k in _CFG_FIELDS if k in raw and raw[k] is not None}
    if "num_key_value_heads" not in kw and "num_attention_heads" in kw:
        kw["num_key_value_heads"] = kw["num_attention_heads"]
    return LlamaConfig(**kw)


def _shard_map(path: str) -> Dict[str, str]:
    """tensor name -> shard file name"""
    idx = os.path.join(path, INDEX)
    if os.path.isfile(idx):
        with open(idx) as f:
            wm = json.load(f)["weight_map"]
        return {k: v for k, v in wm.items()}
    from safetensors import safe_open

    with safe_open(os.path.join(path, SINGLE), framework="pt") as f:
        return {k: SINGLE for k in f.keys()}


def load_hf_weights(model: nn.Module, path: str, strict: bool = True) -> Dict[str, List[str]]:
    """Copy the checkpoint's tensors into ``model``'s parameters / buffers (same names), shard by
    shard.  Returns ``{"loaded", "skipped", "missing"}``; with ``strict`` a missing parameter or an
    unknown tensor raises."""
    from safetensors import safe_open

    targets = dict(model.named_parameters())
    targets.update(dict(model.named_buffers()))
    wmap = _shard_map(path)
    by_file: Dict[str, List[str]] = {}
    for name, fn in wmap.items():
        by_file.setdefault(fn, []).append(name)
    loaded, skipped, unknown = [], [], []
    for fn in sorted(by_file):
        full = os.path.join(path, fn)
        if not fn.endswith(".safetensors"):
            raise ValueError(f"{full}: only safetensors shards are loaded (no pickled checkpoints)")
        with safe_open(full, framework="pt") as f:
            for name in by_file[fn]:
                if name not in targets:
                    (skipped if name.endswith(_SKIP_SUFFIXES) else unknown).append(name)
                    continue
                t = f.get_tensor(name)
                dst = targets[name]
                if tuple(t.shape) != tuple(dst.shape):
                    raise ValueError(f"{name}: checkpoint shape {tuple(t.shape)} != model {tuple(dst.shape)}")
                with torch.no_grad():
                    dst.copy_(t.to(dtype=dst.dtype))
                loaded.append(name)
    tied = getattr(getattr(model, "config", None), "tie_word_embeddings", False)
    missing = [n for n in dict(model.named_parameters()) if n not in set(loaded)
               and not (tied and n == "lm_head.weight")]
    if tied and "lm_head.weight" not in loaded and "model.embed_tokens.weight" in loaded:
        if hasattr(model, "tie_weights"):
            model.tie_weights()  # one shared Parameter (trains as one)
        else:
            with torch.no_grad():
                targets["lm_head.weight"].copy_(targets["model.embed_tokens.weight"])
    if strict and (missing or unknown):
        raise KeyError(f"checkpoint {path}: missing {missing[:8]}{'...' if len(missing) > 8 else ''}, "
                       f"unexpected {unknown[:8]}{'...' if len(unknown) > 8 else ''}")
    return {"loaded": loaded, "skipped": skipped, "missing": missing}


def _config_dict(cfg) -> dict:
    d = {k: getattr(cfg, k) for k in _CFG_FIELDS}
    d.update(architectures=list(getattr(cfg, "architectures", ["LlamaForCausalLM"])), model_type="llama",
             torch_dtype="bfloat16", hidden_act="silu")
    return d


def save_hf_checkpoint(model: nn.Module, path: str, max_shard_bytes: int = 2 << 30,
                       dtype: Optional[torch.dtype] = None) -> List[str]:
    """Write ``model``'s parameters in the HF sharded safetensors layout (+ config.json); returns
    the shard file names.  ``dtype``: cast on the way (e.g. bf16, like HF's Llama-2 release)."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    items: List[Tuple[str, torch.Tensor]] = []
    for name, p in model.named_parameters():
        t = p.detach()
        items.append((name, (t.to(dtype) if dtype is not None else t).contiguous().cpu()))
    shards: List[List[Tuple[str, torch.Tensor]]] = [[]]
    size = 0
    for name, t in items:
        nb = t.numel() * t.element_size()
        if shards[-1] and size + nb > max_shard_bytes:
            shards.append([])
            size = 0
        shards[-1].append((name, t))
        size += nb
    n = len(shards)
    files = []
    wmap = {}
    for i, sh in enumerate(shards):
        fn = SINGLE if n == 1 else f"model-{i + 1:05d}-of-{n:05d}.safetensors"
        save_file({k: v for k, v in sh}, os.path.join(path, fn), metadata={"format": "pt"})
        files.append(fn)
        for k, _ in sh:
            wmap[k] = fn
    if n > 1:
        total = sum(t.numel() * t.element_size() for _, t in items)
        with open(os.path.join(path, INDEX), "w") as f:
            json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, f, indent=1)
    cfg = getattr(model, "config", None)
    if cfg is not None:
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(_config_dict(cfg), f, indent=1)
    return files


def iter_shard_names(path: str) -> Iterable[str]:
    return sorted(set(_shard_map(path).values()))
