#!/bin/bash
# debug-build check + Llama 2-layer op census (which aten ops launch the small kernels)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_debug_build.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1; rc=$?; echo "pytest dbg rc=$rc"; tail -2 gpurun_out/pytest_dbg.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -u scripts/llama_op_profile.py > gpurun_out/llama_census.txt 2>&1; rc=$?; echo "census rc=$rc"; exit $rc
