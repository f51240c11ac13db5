#!/bin/bash
# round 5: LN branch sums in the bias dtype (tests + ViT / GPT-2 graphed steps), CustomTransformer
# fp32 eager host profile (hyperion vs torch kernels)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_llm_ops.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in vitgraph gpt2; do
  timeout -k 10 300 python scripts/run_model_step.py $m > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  grep '^{' $O/$m.log | cut -c1-150
done
for k in hyperion torch; do
  HYPERION_KERNELS=$k timeout -k 10 300 python scripts/eager_host_prof.py ct32 > $O/ct32_$k.log 2>&1 || { tail -5 $O/ct32_$k.log; exit 1; }
  grep "^{" $O/ct32_$k.log
done
