#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_llama_fused.py > gpurun_out/r03w_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03w_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03w_tests.log | head -20; exit $rc; }
for mode in bf16 old bf16 old; do
  HYPERION_WS_PLANS=$mode timeout -k 10 240 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/r03w_llama.log 2>&1; rc=$?
  echo "plans=$mode rc=$rc $(grep '^{' gpurun_out/r03w_llama.log | cut -c90-150)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
