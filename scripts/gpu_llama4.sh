#!/bin/bash
# LoRA one-launch rank-r projection: numerics, Llama-2-7B LoRA graphed step, kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_linear.py tests/test_gpu_llm_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lora.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/run_model_step.py llamagraph > gpurun_out/llamagraph.log 2>&1; rc=$?; echo "graph rc=$rc"; grep "^{" gpurun_out/llamagraph.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace rc=$rc"
