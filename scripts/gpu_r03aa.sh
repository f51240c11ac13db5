#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tiled.py tests/test_gpu_linear.py tests/test_gpu_graph_step.py > gpurun_out/r03aa_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03aa_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03aa_tests.log | head -20; exit $rc; }
for mode in bf16 fp32 bf16 fp32; do
  HYPERION_GEMM_SLAB=$mode timeout -k 10 300 python3 -u scripts/run_model_step.py vitgraph > gpurun_out/r03aa_vit.log 2>&1; rc=$?
  echo "slab=$mode vit rc=$rc $(grep '^{' gpurun_out/r03aa_vit.log | cut -c100-170)"; [ $rc -ne 0 ] && exit $rc
done
for mode in bf16 fp32; do
  HYPERION_GEMM_SLAB=$mode timeout -k 10 300 python3 -u scripts/run_model_step.py gpt2 > gpurun_out/r03aa_gpt2.log 2>&1; rc=$?
  echo "slab=$mode gpt2 rc=$rc $(grep '^{' gpurun_out/r03aa_gpt2.log | cut -c80-170)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
