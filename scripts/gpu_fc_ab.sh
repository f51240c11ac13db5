#!/bin/bash
# ResNet-50 headline with the classifier on hipBLASLt (nn.Linear) vs the native linear ops, A/B/A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for fc in vendor native; do
    HYPERION_RESNET_FC=$fc timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 > gpurun_out/bench_fc_$fc.log 2>&1; rc=$?
    echo "fc=$fc rc=$rc $(tail -1 gpurun_out/bench_fc_$fc.log | cut -c1-130)"; [ $rc -eq 0 ] || exit $rc
  done
done
