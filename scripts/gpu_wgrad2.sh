#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_wgrad.sh || exit $?
timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 > gpurun_out/bench_w0.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_w0.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
HYPERION_WGRAD_STREAM=1 timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 > gpurun_out/bench_w1.log 2>&1; rc=$?; echo "bench side rc=$rc"; tail -1 gpurun_out/bench_w1.log | cut -c1-200
