#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attn_ln.py tests/test_gpu_linear.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ln.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ln.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/gemm_shapes.py --skinny > gpurun_out/skinny.log 2>&1; rc=$?; echo "skinny rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/run_model_step.py llamagraph > gpurun_out/llamagraph.log 2>&1; rc=$?; echo "graph rc=$rc"; grep "^{" gpurun_out/llamagraph.log | cut -c1-200
