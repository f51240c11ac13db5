#!/bin/bash
# LoRA rank-r kernels v2 (written t, pre-zeroed du, vectorized loads): numerics, Llama graphed step,
# kernel trace; staged FSDP capture debug
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_llama_fused.py tests/test_gpu_wstream.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1; rc=$?; echo "lora tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_lora.log | head; tail -1 gpurun_out/pytest_lora.log; fatal $rc
timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_fused.json 2> gpurun_out/llama_fused.err; rc=$?; echo "llama fused rc=$rc"; tail -1 gpurun_out/llama_fused.json | cut -c1-300; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace llama rc=$rc"; fatal $rc
timeout -k 10 240 python3 -u scripts/dbg_fsdp_graph2.py > gpurun_out/dbg_fsdp2.log 2>&1; echo "dbg rc=$?"; grep -v amdgpu gpurun_out/dbg_fsdp2.log | cut -c1-400
