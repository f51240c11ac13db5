#!/bin/bash
# wgrad iteration: numerics tests, then the per-config kernel/reduce probe under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_linear.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or weight or backward or resnet or linear_wgrad" > gpurun_out/pytest_w.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/wprobe" -o run -- python3 scripts/wgrad_probe.py > gpurun_out/wprobe.log 2>&1; rc=$?
echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/wgrad_probe.py --parse gpurun_out/wprobe/run_kernel_trace.csv > gpurun_out/wprobe_parsed.log
echo done
