#!/bin/bash
# round 5: fast GELU backward + act_bwd_colsum grid sweep (ViT / GPT-2 graphed steps)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05y2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py tests/test_gpu_colsum.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in 512 1024 2048; do
  for m in vitgraph gpt2; do
    HYPERION_ACT_COLSUM_WGS=$w timeout -k 10 300 python scripts/run_model_step.py $m > $O/${m}_$w.log 2>&1 || { tail -5 $O/${m}_$w.log; exit 1; }
    echo "wgs=$w $(grep '^{' $O/${m}_$w.log | cut -c1-110)"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/trace_vit" -o run -- python3 "$PWD/scripts/run_model_step.py" vitgraph > $O/vit_trace.log 2>&1 || { tail -5 $O/vit_trace.log; exit 1; }
csv=$(find $O/trace_vit -name '*kernel_trace.csv' | head -1)
python3 scripts/step_trace.py "$csv" --step -2 --out $O/vit_step.txt > /dev/null && rm -f "$csv"
grep -A30 "busy" $O/vit_step.txt | cut -c1-120
