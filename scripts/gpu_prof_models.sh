#!/bin/bash
# rocprofv3 kernel traces of the ViT-B/16 and Llama-2-7B LoRA steps (+ graph-mode timings).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for m in ${*:-vit llama}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_$m" -o run -- python3 "$PWD/scripts/run_model_step.py" $m > gpurun_out/prof_$m.log 2>&1
  rc=$?; echo "$m rc=$rc"; grep '^{' gpurun_out/prof_$m.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
echo done
