#!/bin/bash
# round 5, call O: Llama-2-7B LoRA graphed step — timing + per-step kernel table (rocprofv3 trace)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 400 python scripts/run_model_step.py llamagraph20 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 1; }
grep '^{' $O/llama.log | cut -c1-300
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/trace" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
csv=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/step_trace.py "$csv" --step -2 --out $O/llama_step.txt > /dev/null && grep -n "busy" $O/llama_step.txt && tail -n 40 $O/llama_step.txt
rm -f "$csv"
