#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "[run] $(date +%T) $n"; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[run] $n rc=$rc"; tail -n 4 gpurun_out/$n.log | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
run pytest_gpu 600 python3 -m pytest tests -m gpu -q -x
run hw_bench 600 python3 -m hyperion.cli.hardware_bench --out gpurun_out/hw
echo "[run] done"
