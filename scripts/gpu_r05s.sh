#!/bin/bash
# round 5, call S: LoRA rank-r kernels on a side stream (fused Llama layer) — tests + A/B
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05s; mkdir -p $O
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed" $O/$n.log | tail -2; grep '^{' $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || { tail -25 $O/$n.log; exit $rc; }; }
step pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llama_fused.py
step side1 400 python scripts/run_model_step.py llamagraph20
HYPERION_LORA_STREAM=0 step side0 400 python scripts/run_model_step.py llamagraph20
step side1b 400 python scripts/run_model_step.py llamagraph20
