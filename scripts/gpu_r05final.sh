#!/bin/bash
# round 5 final numbers: bench.py (driver contract) x2, transformer / FSDP / Llama steps
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05final; mkdir -p $O
step() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "[$name] FAILED rc=$?"; tail -8 $O/$name.log; exit 1; }
  echo "[$name] $(grep '^{' $O/$name.log | tail -1 | cut -c1-260)"; }
step bench1 300 python bench.py
step bench2 300 python bench.py
for m in vitgraph vitckptgraph gpt2 lmgraph llamagraph; do step $m 400 python scripts/run_model_step.py $m; done
step fsdp_gpt2_ring3 400 python scripts/run_model_step.py fsdp gpt2_small graph ring3
step fsdp_gpt2_pers 400 python scripts/run_model_step.py fsdp gpt2_small graph
step fsdp_gpt2_coll 400 python scripts/run_model_step.py fsdp gpt2_small graph coll
step fsdp_lm256_coll 400 python scripts/run_model_step.py fsdp lm256 graph coll
