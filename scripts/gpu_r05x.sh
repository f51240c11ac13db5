#!/bin/bash
# round 5, call X: per-kernel PMC table over ResNet-50 steps (5 counter passes) + a graphed step trace
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_suite.sh pmc || exit 1
bash scripts/gpu_r05_trace.sh step_r05x || exit 1
