#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_linear.py tests/test_gpu_llm_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log; fatal $rc
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-160; fatal $rc
timeout -k 10 500 python3 scripts/conv_variants.py fwd,dgrad,wgrad --stages > gpurun_out/conv_variants.log 2>&1; rc=$?; echo "variants rc=$rc"; fatal $rc
echo done
