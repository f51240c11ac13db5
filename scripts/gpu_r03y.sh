#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llama_fused.py > gpurun_out/r03y_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03y_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03y_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r03y_attn.jsonl 2> gpurun_out/r03y_attn.err; rc=$?; cut -c1-150 gpurun_out/r03y_attn.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/run_model_step.py vitgraph > gpurun_out/r03y_vit.log 2>&1; rc=$?; echo "vit rc=$rc $(grep '^{' gpurun_out/r03y_vit.log | cut -c100-200)"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_pmc_attn.sh
