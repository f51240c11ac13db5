#!/bin/bash
# last check of the committed tree: GEMM + debug-build tests, ViT graphed-step kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gemm_tiled.py tests/test_gpu_debug_build.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_last.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_last.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_vit_trace.sh
