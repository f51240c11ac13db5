#!/bin/bash
# A/B of the BN-backward dgrad epilogue per producer kind on the 1-GPU ResNet-50 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for modes in "" "2" "1,2" "0,1,2"; do
  HYPERION_BNB_MODES="$modes" timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 > gpurun_out/ab_bnb.log 2>&1 || exit 1
  echo "modes=[$modes] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bnb.log)"
done
