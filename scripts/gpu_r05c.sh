#!/bin/bash
# round 5, call C: same-box A/B — HEAD (round-4 code, ab_head/) vs the refactored kernels (dual off / dgrad-first)
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2 3; do
  (cd ab_head && timeout -k 10 150 python bench.py --steps 50 --warmup 10) >> gpurun_out/r05/ab_head.jsonl 2>>gpurun_out/r05/ab.err || exit 1
  HYPERION_CONV_DUAL=0 timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/ab_dual0.jsonl 2>>gpurun_out/r05/ab.err || exit 1
  HYPERION_CONV_DUAL=2 timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/ab_dual2.jsonl 2>>gpurun_out/r05/ab.err || exit 1
done
for v in head dual0 dual2; do echo "$v"; python -c "import json,sys; print([json.loads(l)['ms_per_step'] for l in open('gpurun_out/r05/ab_$v.jsonl')])"; done
