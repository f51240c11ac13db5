#!/bin/bash
# transformer steps: tiled GEMM routed by the autotuner (auto) vs vendor only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for m in vitgraph gpt2 lmgraph; do
  for mode in vendor auto; do
    HYPERION_GEMM=$mode timeout -k 10 300 python3 -u scripts/run_model_step.py $m > gpurun_out/step_${m}_$mode.log 2>&1; rc=$?; echo "$m $mode rc=$rc $(grep '^{' gpurun_out/step_${m}_$mode.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
  done
done
