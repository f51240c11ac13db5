#!/bin/bash
# kernel trace of the graphed ResNet-50 bench step (one rocprofv3 --kernel-trace run) + per-step table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-trace}
shift || true
mkdir -p gpurun_out/r05
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/r05/$tag" -o run -- python3 "$PWD/bench.py" --steps 10 --warmup 3 "$@" > gpurun_out/r05/$tag.log 2>&1
rc=$?; echo "trace rc=$rc"; grep '^{' gpurun_out/r05/$tag.log | cut -c1-120
[ $rc -ne 0 ] && exit $rc
csv=$(find gpurun_out/r05/$tag -name '*kernel_trace.csv' | head -1)
python3 scripts/step_trace.py "$csv" --step -2 --out gpurun_out/r05/${tag}_step.txt > /dev/null && tail -n 45 gpurun_out/r05/${tag}_step.txt
rm -f "$csv"
