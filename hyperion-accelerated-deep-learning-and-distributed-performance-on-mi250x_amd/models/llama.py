"""Llama (HF ``LlamaForCausalLM`` key-compatible), random-init, for the LoRA / FSDP fine-tune.

Reference: ``train_llama_fsdp`` loads ``NousResearch/Llama-2-7b-hf`` through HF
``AutoModelForCausalLM`` (``02_development/distributed_utils.py:415-554``; SURVEY C26, §2.5
Llama row: 32 layers, hidden 4096, 32 heads × 128, SwiGLU 11008, RMSNorm, RoPE, V = 32000).
There is no network here, so weights are random-initialised with exactly that architecture
(BASELINE.json: "random-init weights of that architecture"); the state-dict keys equal HF's
(``model.embed_tokens``, ``model.layers.N.self_attn.{q,k,v,o}_proj``,
``model.layers.N.mlp.{gate,up,down}_proj``, ``model.layers.N.{input,post_attention}_layernorm``,
``model.norm``, ``lm_head``), so a real checkpoint loads with ``load_state_dict``.

MI355X path per layer: RMSNorm with the residual add fused (one kernel returns both the normed
activations and the residual stream), q/k/v projections → RoPE applied in place on the
``[B, S, H, 128]`` views by one HIP kernel (``ops.rope``) → causal flash attention with the key
padding mask (``ops.attention``, head_dim 128) → o_proj; SwiGLU as one elementwise kernel
(``ops.swiglu``); the LM head and the shifted cross-entropy are one fused op
(``ops.cross_entropy``).  The FSDP wrap unit is ``LlamaDecoderLayer`` (fixing the reference's
non-recursing policy, K8).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from ..ops import _native
from ..ops import llama_fused as _fused
from ..ops.embedding import Embedding
from ..ops.attention import attention
from ..ops.cross_entropy import LinearCrossEntropy
from ..ops.layernorm import RMSNorm
from ..ops.linear import Linear as HypLinear
from ..ops.rope import apply_rope
from ..ops.swiglu import swiglu


# HYPERION_LLAMA_FUSED=0 keeps every layer on the module path (A/B runs, numerics tests)
FUSED = os.environ.get("HYPERION_LLAMA_FUSED", "1") != "0"


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    initializer_range: float = 0.02
    pad_token_id: Optional[int] = None
    tie_word_embeddings: bool = False
    architectures: List[str] = field(default_factory=lambda: ["LlamaForCausalLM"])

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @classmethod
    def llama2_7b(cls) -> "LlamaConfig":
        return cls()

    @classmethod
    def tiny(cls, **kw) -> "LlamaConfig":
        d = dict(vocab_size=512, hidden_size=128, intermediate_size=344, num_hidden_layers=2,
                 num_attention_heads=2, num_key_value_heads=2, max_position_embeddings=256)
        d.update(kw)
        return cls(**d)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        h, nh, nkv, hd = cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        self.num_heads, self.num_kv, self.head_dim = nh, nkv, hd
        self.q_proj = HypLinear(h, nh * hd, bias=False)
        self.k_proj = HypLinear(h, nkv * hd, bias=False)
        self.v_proj = HypLinear(h, nkv * hd, bias=False)
        self.o_proj = HypLinear(nh * hd, h, bias=False)

    def forward(self, x: torch.Tensor, positions: Optional[torch.Tensor], key_padding_mask: Optional[torch.Tensor]):
        B, S, _ = x.shape
        q = self.q_proj(x).view(B, S, self.num_heads, self.head_dim)
        k = self.k_proj(x).view(B, S, self.num_kv, self.head_dim)
        v = self.v_proj(x).view(B, S, self.num_kv, self.head_dim)
        q, k = apply_rope(q, k, positions, self.cfg.rope_theta)
        if self.num_kv != self.num_heads:  # grouped-query attention: expand K/V heads
            rep = self.num_heads // self.num_kv
            k = k.repeat_interleave(rep, dim=2)
            v = v.repeat_interleave(rep, dim=2)
        o = attention(q, k, v, causal=True, key_padding_mask=key_padding_mask)
        return self.o_proj(o.reshape(B, S, -1))


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_proj = HypLinear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.up_proj = HypLinear(cfg.hidden_size, cfg.intermediate_size, bias=False)
        self.down_proj = HypLinear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.down_proj(swiglu(self.gate_proj(x), self.up_proj(x)))


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.self_attn = LlamaAttention(cfg)
        self.mlp = LlamaMLP(cfg)
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)

    def forward(self, delta: Optional[torch.Tensor], stream: torch.Tensor, positions=None, kpm=None):
        """Residual-stream form: block input = ``stream + delta``; returns ``(mlp_out, new_stream)``.

        Frozen-base layers (the LoRA fine-tune) at few tokens run as ONE fused autograd node
        (``ops/llama_fused.py``: weight-streaming GEMMs over the concatenated q/k/v and gate/up
        weights, LoRA / RoPE / SwiGLU in their epilogues); everything else takes the module path."""
        if positions is None and FUSED:
            out = _fused.llama_layer_fused(self, delta, stream, kpm)
            if out is not None:
                _native.count("llama_fused_layer")
                return out
        ln1 = self.input_layernorm
        if delta is None:
            h, s = ln1(stream), stream
        else:
            h, s = ln1(delta, residual=stream, return_sum=True)
        a = self.self_attn(h, positions, kpm)
        h2, s2 = self.post_attention_layernorm(a, residual=s, return_sum=True)
        return self.mlp(h2), s2

    def block(self, x: torch.Tensor, positions=None, key_padding_mask=None) -> torch.Tensor:
        """Plain form: x -> layer output."""
        d, s = self(None, x, positions, key_padding_mask)
        return s + d


class LlamaModel(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.embed_tokens = Embedding(cfg.vocab_size, cfg.hidden_size, padding_idx=cfg.pad_token_id)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.gradient_checkpointing = False

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        x = self.embed_tokens(input_ids)
        kpm = None
        positions = None
        if attention_mask is not None:
            # nonzero = padded key; uint8 once per forward (the kernels' mask dtype) instead of a
            # bool -> uint8 copy in each of the 32 layers
            kpm = (attention_mask == 0).to(torch.uint8)
            # HF computes positions from the mask only when generating; training uses arange
        d: Optional[torch.Tensor] = None
        s = x
        ckpt = self.gradient_checkpointing and self.training and torch.is_grad_enabled()
        for layer in self.layers:
            if ckpt:
                d, s = checkpoint(layer, d, s, positions, kpm, use_reentrant=False)
            else:
                d, s = layer(d, s, positions, kpm)
        return self.norm(d, residual=s) if d is not None else self.norm(s)


class CausalLMOutput(dict):
    """Minimal HF-style output (``.loss``, ``.logits``)."""

    __getattr__ = dict.get


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: Optional[LlamaConfig] = None):
        super().__init__()
        self.config = cfg or LlamaConfig()
        self.model = LlamaModel(self.config)
        self.lm_head = LinearCrossEntropy(self.config.hidden_size, self.config.vocab_size, bias=False)
        self.apply(self._init_weights)
        if self.config.tie_word_embeddings:
            self.tie_weights()

    def tie_weights(self) -> None:
        """HF ``tie_word_embeddings``: ONE Parameter serves as the input embedding and the LM head,
        so both train together (a copy would drift apart after the first optimizer step)."""
        self.lm_head.weight = self.model.embed_tokens.weight

    def _init_weights(self, m: nn.Module) -> None:
        std = self.config.initializer_range
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=std)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=std)

    def gradient_checkpointing_enable(self) -> None:
        self.model.gradient_checkpointing = True

    @classmethod
    def from_pretrained(cls, path: str, torch_dtype: Optional[torch.dtype] = None,
                        device: Optional[torch.device] = None, config: Optional[LlamaConfig] = None,
                        strict: bool = True) -> "LlamaForCausalLM":
        """A LOCAL HF checkpoint directory (config.json + safetensors shards; models/hf_checkpoint.py):
        the reference's ``AutoModelForCausalLM.from_pretrained`` without the network.  Weights-only
        loading, tensor by tensor into the built model."""
        from .hf_checkpoint import load_hf_weights, load_llama_config

        cfg = config or load_llama_config(path)
        with torch.device(device or "cpu"):
            m = cls(cfg)
        if torch_dtype is not None:
            m = m.to(torch_dtype)
        load_hf_weights(m, path, strict=strict)
        if cfg.tie_word_embeddings:
            m.tie_weights()
        return m

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None, return_logits: Optional[bool] = None) -> CausalLMOutput:
        h = self.model(input_ids, attention_mask)
        out = CausalLMOutput()
        if labels is not None:
            # HF semantics: predict labels[:, 1:] from positions [:, :-1]; -100 is ignored
            hs = h[:, :-1]
            tgt = labels[:, 1:].contiguous()
            out["loss"] = self.lm_head(hs, target=tgt, ignore_index=-100)
        if return_logits or (return_logits is None and labels is None):
            out["logits"] = self.lm_head(h)
        return out


def llama2_7b(**kw) -> LlamaForCausalLM:
    return LlamaForCausalLM(LlamaConfig.llama2_7b())


def param_count(cfg: LlamaConfig) -> int:
    h, i, v, L = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size, cfg.num_hidden_layers
    kv = cfg.num_key_value_heads * cfg.head_dim
    per_layer = h * h * 2 + h * kv * 2 + 3 * h * i + 2 * h
    return L * per_layer + 2 * v * h + h

