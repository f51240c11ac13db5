#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_graph_step.py tests/test_gpu_fsdp_graph.py > gpurun_out/r03x_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03x_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03x_tests.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u scripts/run_model_step.py vitgraph > gpurun_out/r03x_vit.log 2>&1; rc=$?; echo "vit rc=$rc $(grep '^{' gpurun_out/r03x_vit.log | cut -c1-200)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/run_model_step.py lmgraph > gpurun_out/r03x_lm.log 2>&1; rc=$?; echo "lm rc=$rc $(grep '^{' gpurun_out/r03x_lm.log | cut -c1-200)"; [ $rc -ne 0 ] && exit $rc
exit 0
