#!/bin/bash
# kernel traces of two run_model_step.py invocations: gpu_trace_pair.sh "<args A>" "<args B>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for args in "$@"; do
  rm -rf gpurun_out/trace_pair$i
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_pair$i" -o run -- python3 "$PWD/scripts/run_model_step.py" $args > gpurun_out/trace_pair$i.log 2>&1; rc=$?
  echo "[$args] rc=$rc"; grep '^{' gpurun_out/trace_pair$i.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
