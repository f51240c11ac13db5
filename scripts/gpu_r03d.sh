#!/bin/bash
# Llama-2-7B LoRA graphed step: fused layer vs module path, and a kernel trace of the fused step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_llama_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1; rc=$?; echo "fused tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_fused.log | head; tail -1 gpurun_out/pytest_fused.log; fatal $rc
timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_fused.json 2> gpurun_out/llama_fused.err; rc=$?; echo "llama fused rc=$rc"; tail -1 gpurun_out/llama_fused.json | cut -c1-300; fatal $rc
HYPERION_LLAMA_FUSED=0 timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_module.json 2> gpurun_out/llama_module.err; rc=$?; echo "llama module rc=$rc"; tail -1 gpurun_out/llama_module.json | cut -c1-300; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace rc=$rc"
