#!/bin/bash
# ViT iteration: linear/LN tests, ViT-B/16 step (no ckpt + ckpt), op census.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[$n] rc=$rc"; grep -E "passed|failed|^\{" gpurun_out/$n.log | cut -c1-260 | tail -3; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$n.log; exit $rc; fi; }
run pytest 300 python3 -u -m pytest tests/test_gpu_linear.py tests/test_gpu_attn_ln.py tests/test_gpu_llm_ops.py -x -q --timeout 120 --timeout-method thread
run vit 300 python3 scripts/run_model_step.py vit
run vitckpt 300 python3 scripts/run_model_step.py vitckpt
timeout -k 10 240 python3 scripts/op_census.py vit > gpurun_out/vit_ops.txt 2>&1; echo "census rc=$?"
