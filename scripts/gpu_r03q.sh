#!/bin/bash
# kernel traces: GPT-2-small graphed step, plain vs FSDP world 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
rm -rf gpurun_out/trace_gpt2 gpurun_out/trace_gpt2fsdp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_gpt2" -o run -- python3 "$PWD/scripts/run_model_step.py" gpt2 > gpurun_out/trace_gpt2.log 2>&1; rc=$?; echo "gpt2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_gpt2fsdp" -o run -- python3 "$PWD/scripts/run_model_step.py" fsdp gpt2_small graph > gpurun_out/trace_gpt2fsdp.log 2>&1; rc=$?; echo "gpt2 fsdp rc=$rc"
exit $rc
