#!/bin/bash
# Linear/LoRA kernel numerics, then Llama-2-7B LoRA step (graph) + op census.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_linear.py tests/test_gpu_llm_ops.py tests/test_gpu_attn_ln.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_linear.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_linear.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 scripts/run_model_step.py llamagraph > gpurun_out/llamagraph.log 2>&1
rc=$?; echo "llamagraph rc=$rc"; grep '^{' gpurun_out/llamagraph.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python3 scripts/llama_op_profile.py > gpurun_out/llama_ops.txt 2>&1; echo "ops rc=$?"
