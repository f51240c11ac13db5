#!/bin/bash
# tiled GEMM numerics + debug build check + shape bench (hipGraph timing)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gemm_tiled.py tests/test_gpu_debug_build.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/gemm_tiled_bench.py --sweep --out gpurun_out/gemm_tiled.json > gpurun_out/gemm_tiled.log 2>&1; rc=$?; echo "bench rc=$rc"; exit $rc
