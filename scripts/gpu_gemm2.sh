#!/bin/bash
# tiled GEMM: numerics tests, shape benchmark + sweep, transformer steps with the tiled kernel routed (auto) vs vendor
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm_tiled.py tests/test_gpu_linear.py tests/test_gpu_llm_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/gemm_tiled_bench.py --sweep --out gpurun_out/gemm_tiled.json > gpurun_out/gemm_tiled.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
for mode in vendor auto; do
  for m in vitgraph gpt2 lmgraph; do
    HYPERION_GEMM=$mode timeout -k 10 300 python3 -u scripts/run_model_step.py $m > gpurun_out/step_${m}_$mode.log 2>&1; rc=$?; echo "$m $mode rc=$rc $(grep '^{' gpurun_out/step_${m}_$mode.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
  done
done
