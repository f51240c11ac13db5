#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wstream.py tests/test_gpu_llama_fused.py > gpurun_out/r03u_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03u_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/r03u_tests.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 240 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/r03u_llama.log 2>&1; rc=$?
  echo "run $i rc=$rc $(grep '^{' gpurun_out/r03u_llama.log | cut -c1-160)"; [ $rc -ne 0 ] && exit $rc
done
rm -rf gpurun_out/trace_llama
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace rc=$rc"
exit $rc
