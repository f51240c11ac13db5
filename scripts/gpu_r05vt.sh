#!/bin/bash
# round 5: per-step kernel table of the graphed ViT-B/16 and GPT-2 steps
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05vt; mkdir -p $O
for m in vitgraph gpt2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/trace_$m" -o run -- python3 "$PWD/scripts/run_model_step.py" $m > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  grep '^{' $O/$m.log | cut -c1-120
  csv=$(find $O/trace_$m -name '*kernel_trace.csv' | head -1)
  python3 scripts/step_trace.py "$csv" --step -2 --out $O/${m}_step.txt > /dev/null || exit 1
  rm -f "$csv"
  grep -A25 "busy" $O/${m}_step.txt | cut -c1-120
done
