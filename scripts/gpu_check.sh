#!/bin/bash
# GPU-box check: smoke, GPU tests, benches (A/B), rocprofv3 kernel-trace profiles.
# Every GPU step runs under its own timeout; a crash/abort/timeout ends the script.
# Usage: bash scripts/gpu_check.sh [steps...]
#   steps: smoke tests bench eager torch prof proftorch   (default: smoke tests bench eager prof)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${*:-smoke tests bench eager prof}

run_step() {
  local name=$1 t=$2
  shift 2
  echo "[gpu_check] $(date +%T) start $name"
  timeout -k 10 "$t" "$@" >"gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_check] $(date +%T) $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[gpu_check] fatal rc=$rc in $name; stopping"
    exit $rc
  fi
}

for s in $STEPS; do
  case $s in
    smoke) run_step smoke 300 python3 __graft_entry__.py smoke ;;
    tests) run_step pytest_gpu 600 python3 -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread ;;
    bench) run_step bench_graph 400 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json ;;
    eager) run_step bench_eager 400 python3 bench.py --steps 30 --warmup 10 --graph 0 --json-out gpurun_out/bench_eager.json ;;
    torch)
      run_step bench_torch_eager 400 python3 bench.py --steps 30 --warmup 10 --graph 0 --kernels torch --amp autocast --json-out gpurun_out/bench_torch_eager.json
      run_step bench_torch_graph 400 python3 bench.py --steps 30 --warmup 10 --graph 1 --kernels torch --amp autocast --json-out gpurun_out/bench_torch_graph.json ;;
    prof) run_step prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_bench" -o run -- python3 "$PWD/bench.py" --steps 10 --warmup 5 --graph 0 ;;
    proftorch) run_step prof_torch 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_torch" -o run -- python3 "$PWD/bench.py" --steps 10 --warmup 5 --graph 0 --kernels torch --amp autocast ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "[gpu_check] done"
