#!/bin/bash
# round 5, call V: conv plans re-tuned (+ the fused launch's weight-gradient split-K and grid order) with every data gradient timed INSIDE the fused dgrad+wgrad
# launch (and the forward with write-through stores); bench A/B default plans vs the new table
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 900 python -u scripts/conv_tune.py --dual --out $O/conv_plans_dual.json --raw $O/conv_tune_dual_raw.json > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
tail -5 $O/tune.log
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> $O/bench_default.jsonl 2>>$O/bench.err || exit 1
  HYPERION_CONV_PLANS=$O/conv_plans_dual.json timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> $O/bench_dual.jsonl 2>>$O/bench.err || exit 1
done
python -c "
import json
for f in ['$O/bench_default.jsonl','$O/bench_dual.jsonl']:
    print(f, [json.loads(l)['ms_per_step'] for l in open(f)])
"
