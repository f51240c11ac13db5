#!/bin/bash
# Round-2 GPU call C: per-kernel step trace of the headline bench, vendor-GEMM reference times for
# every conv's GEMM shape, STREAM launch-mode / unroll sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_bench" -o run -- python3 "$PWD/bench.py" --steps 6 --warmup 4 > gpurun_out/trace_bench.log 2>&1; rc=$?; echo "trace rc=$rc"; fatal $rc
timeout -k 10 300 python3 scripts/conv_gemm_equiv.py > gpurun_out/conv_gemm_equiv.log 2>&1; rc=$?; echo "gemm equiv rc=$rc"; fatal $rc
timeout -k 10 200 python3 scripts/hw_one.py sweep > gpurun_out/stream_sweep.log 2>&1; rc=$?; echo "sweep rc=$rc"; fatal $rc
echo done
