#!/bin/bash
# round 5, call M: split-K last arriver (GEMM tests, probe A/B, GPT-2 / ViT A/B), FSDP ring capture
# tests + GPT-2 FSDP ring vs persistent, stem one-launch transforms, empty-segment skipping
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05m; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" $O/$n.log | cut -c1-300 | tail -3; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_tiled.py tests/test_gpu_linear.py tests/test_gpu_gemm.py tests/test_gpu_round4.py tests/test_gpu_fsdp_graph.py tests/test_gpu_ddp_graph.py
step probe_inkernel 400 python scripts/gemm_probe.py --out $O/probe_inkernel.json
HYPERION_SPLITK_INKERNEL=0 step probe_separate 400 python scripts/gemm_probe.py --out $O/probe_separate.json
python - <<PY
import json
a=json.load(open('$O/probe_inkernel.json')); b=json.load(open('$O/probe_separate.json'))
for x,y in zip(a,b):
    ks=[k for k in x if k.startswith('t2_s') and k not in ('t2_s1','t2_s-1')]
    print(x['shape'], 'best in', x['native_best'], 'sep', y['native_best'], 'vendor', x['vendor_us'], x['vendor_gemm_only_us'], {k:(x[k], y.get(k)) for k in ks})
PY
step gpt2_in 300 python scripts/run_model_step.py gpt2
HYPERION_SPLITK_INKERNEL=0 step gpt2_sep 300 python scripts/run_model_step.py gpt2
step vit_in 300 python scripts/run_model_step.py vitgraph
HYPERION_SPLITK_INKERNEL=0 step vit_sep 300 python scripts/run_model_step.py vitgraph
step bench 150 python bench.py --steps 50 --warmup 10
step bench_fusedloss 150 python bench.py --steps 50 --warmup 10 --loss fused
step fsdp_gpt2_persist 300 python scripts/run_model_step.py fsdp gpt2_small graph
step fsdp_gpt2_ring3 300 python scripts/run_model_step.py fsdp gpt2_small graph ring3
step fsdp_gpt2_ring3_coll 300 python scripts/run_model_step.py fsdp gpt2_small graph ring3 coll
step fsdp_gpt2_persist_coll 300 python scripts/run_model_step.py fsdp gpt2_small graph coll
step fsdp_lm_coll 300 python scripts/run_model_step.py fsdp lm256 graph coll
