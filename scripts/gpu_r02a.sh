#!/bin/bash
# Round-2 GPU call A: smoke, full GPU test suite, headline bench. Each step under its own timeout;
# a crash / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local name=$1 t=$2; shift 2
  echo "[r02a] $(date +%T) start $name"
  timeout -k 10 "$t" "$@" >"gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[r02a] $(date +%T) $name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[r02a] fatal rc=$rc in $name"; exit $rc; fi
}
step smoke 300 python3 __graft_entry__.py smoke
step bench 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json
step pytest_gpu 800 python3 -u -m pytest tests -m gpu -v -rf -x --timeout 120 --timeout-method thread
echo "[r02a] done"
