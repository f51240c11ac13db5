#!/bin/bash
# kernel trace of the graphed ViT-B/16 step (tiled GEMM routed by the autotuner)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_vit" -o run -- python3 "$PWD/scripts/run_model_step.py" vitgraph > gpurun_out/trace_vit.log 2>&1; rc=$?; echo "trace rc=$rc"; grep '^{' gpurun_out/trace_vit.log | cut -c1-160
