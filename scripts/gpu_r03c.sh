#!/bin/bash
# fused Llama layer tests + weight-streaming sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wstream.py tests/test_gpu_llama_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ws.log 2>&1; rc=$?; echo "ws tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_ws.log | head -20; tail -2 gpurun_out/pytest_ws.log; fatal $rc
timeout -k 10 400 python3 -u scripts/ws_bench.py > gpurun_out/ws_bench.log 2>&1; rc=$?; echo "ws bench rc=$rc"; grep -v amdgpu.ids gpurun_out/ws_bench.log | cut -c1-400; fatal $rc
