"""Run one model step benchmark (for rocprofv3 kernel traces): python scripts/run_model_step.py {vit,llama,lm,gpt2}"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hyperion.bench import models as M  # noqa: E402

which = sys.argv[1]
if which == "fsdp":  # fsdp <lm256|gpt2_small|llama7b_lora> [graph] [shardbase] [coll] [reshard]
    model = sys.argv[2]
    kw = dict(graph="graph" in sys.argv[3:], collectives_at_world_1="coll" in sys.argv[3:])
    if "reshard" in sys.argv[3:]:
        kw["persistent"] = False
    for a in sys.argv[3:]:
        if a.startswith("ring"):  # ring2 / ring3: FULL_SHARD ring of gathered-unit slots
            kw["ring"] = int(a[4:])
    if "shardbase" in sys.argv[3:]:
        kw["replicate_frozen"] = False
    if model == "gpt2_small":
        kw["batch"] = 16
    if model.startswith("llama7b"):
        kw["batch"] = 1
    if "curve" in sys.argv[3:]:
        kw["loss_curve"] = True
    steps = 50 if model == "llama7b_full" else 10
    r = M.bench_fsdp_step(model, steps=steps, warmup=3, **kw)
elif which == "vit":
    r = M.bench_vit_step(checkpointing=False, steps=5, warmup=3)
elif which == "vitgraph":
    r = M.bench_vit_step(checkpointing=False, steps=20, warmup=5, graph=True)
elif which == "vitckptgraph":
    r = M.bench_vit_step(checkpointing=True, steps=20, warmup=5, graph=True)
elif which == "vitselgraph":
    r = M.bench_vit_step(checkpointing="selective", steps=20, warmup=5, graph=True)
elif which == "vitckpt":
    r = M.bench_vit_step(checkpointing=True, steps=5, warmup=3)
elif which == "llama":
    r = M.bench_llama_lora_step(steps=3, warmup=2, graph=False)
elif which == "llama1":  # one warm-up + one timed eager step (PMC passes: small counter files)
    r = M.bench_llama_lora_step(steps=1, warmup=1, graph=False)
elif which == "llamagraph":
    r = M.bench_llama_lora_step(steps=5, warmup=3, graph=True)
elif which == "llamagraph20":
    r = M.bench_llama_lora_step(steps=20, warmup=3, graph=True)
elif which == "lmddp1":  # LM-256 graphed under DDP(buckets_at_world_1, NativeComm)
    r = M.bench_lm_step(precision="bf16", graph=True, steps=20, warmup=5, ddp_world1=True)
elif which == "lmddp1g":  # ... as ONE graph with the RCCL all-reduces captured
    r = M.bench_lm_step(precision="bf16", graph=True, steps=20, warmup=5, ddp_world1=True, one_graph=True)
elif which == "vitddp1g":
    r = M.bench_vit_step(checkpointing=False, steps=20, warmup=5, graph=True, ddp_world1=True, one_graph=True)
elif which == "vitddp1":
    r = M.bench_vit_step(checkpointing=False, steps=20, warmup=5, graph=True, ddp_world1=True)
elif which == "lmgraph":
    r = M.bench_lm_step(precision="bf16", graph=True, steps=20, warmup=5)
elif which == "lm":
    r = M.bench_lm_step(precision="bf16", steps=5, warmup=3)
else:
    r = M.bench_lm_step(precision="bf16", graph=True, model="gpt2_small", batch=16, steps=10, warmup=3)
if which in ("gpt2", "lmgraph", "lm", "vit", "vitgraph", "vitckptgraph", "vitselgraph"):
    from hyperion.ops import gemm as _gemm

    r["gemm_choices"] = {"x".join(map(str, k)): v for k, v in _gemm.choices().items()}
print(json.dumps(r), flush=True)
