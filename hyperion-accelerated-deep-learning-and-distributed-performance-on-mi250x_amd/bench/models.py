"""Training-step throughput of the LM / ViT / Llama configs on one GPU (BASELINE.json configs 3-5).

Each function builds the model exactly as the matching trainer does, runs ``warmup`` steps, then
times ``steps`` full steps (forward, backward, optimizer) between device syncs, and returns
samples/s, tokens/s, ms/step and peak memory.  Used by ``cli/bench_models`` and the profiling runs.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, Optional

import torch


def _timeit(step, steps: int, warmup: int) -> float:
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def bench_lm_step(batch: int = 32, seq: int = 128, precision: str = "fp16", steps: int = 20, warmup: int = 5,
                  model: str = "lm256", causal: bool = False, graph: bool = False,
                  compute_copies: Optional[bool] = None, ddp_world1: bool = False, one_graph: bool = False) -> Dict:
    """SimpleTransformerLM (C14) training step as in train_language_model_ddp (single GPU).
    ``compute_copies`` (default for bf16): the parameters live in bf16 with fp32 masters inside
    FusedAdam (train.amp.cast_for_compute, as the ViT bench) instead of fp32 parameters cast by
    autocast on every step; fp16 keeps the reference's autocast + loss-scaler methodology."""
    from ..data.synthetic import SyntheticWikiText2
    from ..models.simple_lm import GPT2_PAD, gpt2_small_lm, simple_lm_256
    from ..ops.optim import FusedAdam
    from ..train.amp import LossScaler

    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = (simple_lm_256(causal=causal) if model == "lm256" else gpt2_small_lm()).to(dev)
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[precision]
    copies = (precision == "bf16") if compute_copies is None else bool(compute_copies and dt is not None)
    if copies:
        from ..train.amp import cast_for_compute

        cast_for_compute(m, dt)
    dpm = _ddp_world1(m) if ddp_world1 else None
    opt = FusedAdam(m.parameters(), lr=2e-4, weight_decay=0.01, adamw=True, zero_grad_in_step=graph)
    scaler = LossScaler(enabled=precision == "fp16", device=dev)
    ids = SyntheticWikiText2(n=batch, seq_len=seq, seed=0).input_ids.to(dev)
    x, y = ids[:, :-1].contiguous(), ids[:, 1:].contiguous()

    def body():
        opt.zero_grad(set_to_none=not graph)
        with torch.autocast("cuda", dtype=dt or torch.float32, enabled=dt is not None and not copies):
            loss = m.forward_loss(x, y, ignore_index=GPT2_PAD)
        if scaler.enabled:
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
        else:
            loss.backward()
            opt.step()
        return loss.detach()

    step = _graphed(body, m, dpm, one_graph) if graph else body
    torch.cuda.reset_peak_memory_stats()
    t = _timeit(step, steps, warmup)
    return {"model": model, "batch": batch, "seq": seq, "precision": precision, "graph": graph,
            "compute_copies": copies, "ms_per_step": t * 1e3, **_ddp_info(dpm), "one_graph": one_graph,
            "samples_per_s": batch / t, "tokens_per_s": batch * (seq - 1) / t,
            "peak_mem_mb": torch.cuda.max_memory_allocated() / 2**20}


def bench_vit_step(batch: int = 32, precision: str = "bf16", checkpointing: bool = True, steps: int = 20,
                   warmup: int = 5, graph: bool = False, ddp_world1: bool = False, one_graph: bool = False) -> Dict:
    """ViT-B/16 bf16 + activation checkpointing (BASELINE.json config 3), MSE/Adam like C6.
    ``graph``: the whole step captured once as a hipGraph and replayed."""
    from ..models.vit import vit_b_16
    from ..ops.optim import FusedAdam
    from ..train.amp import cast_for_compute

    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = vit_b_16(use_checkpoint=checkpointing).to(dev).to(memory_format=torch.channels_last)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(precision)
    if dt is not None:
        cast_for_compute(m, dt)
    dpm = _ddp_world1(m) if ddp_world1 else None
    opt = FusedAdam(m.parameters(), lr=1e-3, zero_grad_in_step=graph)
    x = torch.rand(batch, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    x = x.to(dt) if dt is not None else x
    y = torch.rand(batch, 1000, device=dev)

    def body():
        opt.zero_grad(set_to_none=not graph)
        loss = torch.nn.functional.mse_loss(m(x).float(), y)
        loss.backward()
        opt.step()
        return loss.detach()

    step = _graphed(body, m, dpm, one_graph) if graph else body
    torch.cuda.reset_peak_memory_stats()
    t = _timeit(step, steps, warmup)
    return {"model": "vit_b_16", "batch": batch, "precision": precision, "checkpointing": checkpointing,
            "graph": graph, "ms_per_step": t * 1e3, "samples_per_s": batch / t, **_ddp_info(dpm),
            "peak_mem_mb": torch.cuda.max_memory_allocated() / 2**20}


def bench_llama_lora_step(batch: int = 1, seq: int = 128, steps: int = 10, warmup: int = 3, lora: bool = True,
                          config=None, grad_ckpt: bool = False, graph: bool = True) -> Dict:
    """Llama-2-7B (random init) LoRA r16 bf16 step, batch 1 x 128 tokens (the reference's Llama run)."""
    from ..data.synthetic import SyntheticWikiText2
    from ..models.llama import LlamaConfig, LlamaForCausalLM
    from ..models.lora import apply_lora, trainable_parameters
    from ..ops.optim import FusedAdam

    dev = torch.device("cuda")
    torch.manual_seed(0)
    cfg = config or LlamaConfig.llama2_7b()
    with torch.device(dev):
        m = LlamaForCausalLM(cfg).to(torch.bfloat16)
    if lora:
        apply_lora(m)
    if grad_ckpt:
        m.gradient_checkpointing_enable()
    params = [p for p in m.parameters() if p.requires_grad]
    opt = FusedAdam(params, lr=1e-5, weight_decay=0.01, adamw=True, zero_grad_in_step=graph)
    ds = SyntheticWikiText2(n=batch, seq_len=seq, seed=0)
    ids = (ds.input_ids % cfg.vocab_size).to(dev)
    mask = ds.attention_mask.to(dev)

    from ..ops.optim import clip_grad_norm_
    from ..train.step import GraphedClosure

    def body():
        opt.zero_grad(set_to_none=not graph)
        loss = m(ids, attention_mask=mask, labels=ids).loss
        loss.backward()
        clip_grad_norm_(params, 1.0)
        opt.step()
        return loss.detach()

    step = GraphedClosure(body, warmup=2, module=m) if graph else body
    torch.cuda.reset_peak_memory_stats()
    t = _timeit(step, steps, warmup)
    return {"model": "llama2_7b" if config is None else "llama_custom", "lora": lora, "graph": graph, "batch": batch,
            "seq": seq,
            "ms_per_step": t * 1e3, "samples_per_s": batch / t, "tokens_per_s": batch * seq / t,
            "trainable_params": trainable_parameters(m), "peak_mem_mb": torch.cuda.max_memory_allocated() / 2**20}




def _ddp_world1(m):
    """m's parameters under Hyperion DDP on one GPU: buckets on, native RCCL communicator.
    HYPERION_DDP_COMM_DTYPE=param reduces in the parameters' dtype (torch DDP's semantics: the
    gradients then live in their bucket slots, no pack copies); default fp32 buckets."""
    from ..parallel import DDP
    from ..parallel.comm import NativeComm

    _ensure_pg()
    dev = next(m.parameters()).device
    kw = {"comm_dtype": None} if os.environ.get("HYPERION_DDP_COMM_DTYPE") == "param" else {}
    return DDP(m, buckets_at_world_1=True, comm=NativeComm(dev), broadcast_buffers=False, **kw)


def _graphed(body, m, dpm, one_graph: bool = False):
    """The step as one hipGraph — or, under DDP, as graph segments with the bucket all-reduces as
    eager holes (train/segments.py: the trainers' capture of a data-parallel step).  one_graph:
    DDP too as ONE graph, the native RCCL all-reduces recorded into it (stream fork / join)."""
    if dpm is not None and not one_graph:
        from ..train.segments import SegmentedStep

        return SegmentedStep(body, warmup=2, module=m)
    from ..train.step import GraphedClosure

    return GraphedClosure(body, warmup=2, module=m)


def _ddp_info(dpm) -> Dict:
    if dpm is None:
        return {}
    return {"ddp_world1": True, "comm": type(dpm.comm).__name__, "buckets": len(dpm.bucket_sizes())}



def _ensure_pg() -> None:
    """A world-1 RCCL process group when none is up (FSDP's collectives need one; under
    ``torch.distributed.run`` the launcher's group is used as is)."""
    import os
    import socket

    import torch.distributed as dist

    if dist.is_initialized():
        return
    if "MASTER_PORT" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", rank=int(os.environ.get("RANK", 0)), world_size=int(os.environ.get("WORLD_SIZE", 1)),
                            device_id=torch.device("cuda", torch.cuda.current_device()))


def bench_fsdp_step(model: str = "lm256", batch: int = 32, seq: int = 128, steps: int = 10, warmup: int = 3,
                    graph: bool = False, replicate_frozen="auto", persistent=None,
                    collectives_at_world_1: bool = False, loss_curve: bool = False, lr: float = 1e-4,
                    ring: int = 0) -> Dict:
    """One FSDP FULL_SHARD training step exactly as the FSDP trainers run it (C25 / BASELINE config
    4 / C26): Hyperion's FSDP over the native RCCL communicator, bf16 mixed precision (param /
    reduce / buffer), FusedAdamW, global-norm clip 1.0.  ``model``: ``lm256`` (size-based wrap,
    100k params), ``gpt2_small`` (one unit per transformer layer), ``llama7b_lora`` (LoRA r16,
    one unit per decoder layer, frozen base weights sharded too).  World size = the launcher's
    (1 on a single GPU: the gathers / reduce-scatters are then identity collectives, but every
    flat-buffer pack, cast and hook runs).  ``graph=True``: the step is captured once as graph
    segments with the collectives as eager holes (``train/segments.py``; persistent FSDP buffers, or
    with ``ring`` >= 2 the FULL_SHARD ring of fixed-address gathered-unit slots)."""
    import torch.distributed as dist

    from ..data.synthetic import SyntheticWikiText2
    from ..ops.optim import FusedAdam
    from ..parallel.fsdp import FSDP, MixedPrecision, size_based_auto_wrap_policy, transformer_auto_wrap_policy

    _ensure_pg()
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    bf = torch.bfloat16
    if model in ("llama7b_lora", "llama7b_full"):
        from ..models.llama import LlamaConfig, LlamaDecoderLayer, LlamaForCausalLM
        from ..models.lora import apply_lora

        cfg = LlamaConfig.llama2_7b()
        with torch.device(dev):
            base = LlamaForCausalLM(cfg).to(bf)
        if model == "llama7b_lora":
            apply_lora(base)
        policy = transformer_auto_wrap_policy({LlamaDecoderLayer})
        vocab = cfg.vocab_size
    else:
        from ..models.simple_lm import GPT2_PAD, gpt2_small_lm, simple_lm_256
        from ..models.transformer import TransformerEncoderLayer

        base = simple_lm_256() if model == "lm256" else gpt2_small_lm()
        policy = (size_based_auto_wrap_policy(100_000) if model == "lm256"
                  else transformer_auto_wrap_policy({TransformerEncoderLayer}))
        vocab = 50257
    m = FSDP(base, auto_wrap_policy=policy, device_id=dev, mixed_precision=MixedPrecision(bf, bf, bf),
             replicate_frozen=replicate_frozen if model == "llama7b_lora" else False,
             persistent=(True if graph and not ring else persistent), collectives_at_world_1=collectives_at_world_1,
             ring=ring)
    params = [p for p in m.parameters() if p.requires_grad]
    opt = FusedAdam(params, lr=lr, weight_decay=0.01, adamw=True)
    ds = SyntheticWikiText2(n=batch, seq_len=seq, seed=dist.get_rank())
    ids = (ds.input_ids % vocab).to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        if model.startswith("llama7b"):
            loss = m(ids, labels=ids).loss
        else:
            # FSDP's MixedPrecision already holds the gathered parameters in bf16: no autocast (its
            # per-op fp32 casts of bf16 activations and weights were ~0.5 ms of the GPT-2 step)
            loss = m.forward_loss(ids[:, :-1], ids[:, 1:], ignore_index=GPT2_PAD)
        loss.backward()
        m.clip_grad_norm_(1.0, defer_to=opt)  # the coefficient is applied inside the Adam kernel
        opt.step()
        return loss.detach()

    seg = None
    if graph:
        from ..train.segments import SegmentedStep

        seg = SegmentedStep(step, warmup=2, module=m)
    torch.cuda.reset_peak_memory_stats()
    run = seg if seg is not None else step
    curve = []

    def timed():
        out = run()
        if loss_curve:
            curve.append(out.detach().clone().reshape(()))  # (a graphed step returns one static tensor)
        return out

    t = _timeit(timed if loss_curve else run, steps, warmup)
    final_loss = float(run())  # one more step: the timed schedule trains
    if not math.isfinite(final_loss):
        raise RuntimeError(f"bench_fsdp_step({model}, graph={graph}): non-finite loss {final_loss}")
    world = dist.get_world_size()
    tok = batch * (seq if model.startswith("llama7b") else seq - 1)
    return {"model": model, "fsdp": True, "world": world, "graph": graph, "persistent": m.persistent,
            "ring": m.ring, "memory_plan": m.memory_plan(),
            "persistent_reason": m.persistent_reason, "collectives_at_world_1": collectives_at_world_1,
            "comm": type(m.comm).__name__,
            "replicate_frozen": m.replicate_frozen,
            "segments": seg.seg.num_segments if seg is not None and seg.seg is not None else 0,
            "batch_per_gpu": batch, "seq": seq, "ms_per_step": t * 1e3,
            "samples_per_s": world * batch / t, "tokens_per_s": world * tok / t,
            "trainable_params": sum(p.numel() for p in params), "peak_mem_mb": torch.cuda.max_memory_allocated() / 2**20,
            "final_loss": final_loss,
            **({"loss_curve": [round(v, 4) for v in torch.stack(curve[warmup:]).tolist()]} if loss_curve else {})}
