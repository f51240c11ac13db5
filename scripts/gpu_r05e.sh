#!/bin/bash
# round 5, call E: write-through (sc1) output stores vs plain (ab_head/ = the same tree built with HYP_WT_STORES=0)
set -o pipefail
mkdir -p gpurun_out/r05
for i in 1 2 3; do
  (cd ab_head && timeout -k 10 150 python bench.py --steps 50 --warmup 10) >> gpurun_out/r05/wt_plain.jsonl 2>>gpurun_out/r05/wt.err || exit 1
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/wt_sc1.jsonl 2>>gpurun_out/r05/wt.err || exit 1
done
for v in plain sc1; do echo "$v"; python -c "import json,sys; print([json.loads(l)['ms_per_step'] for l in open('gpurun_out/r05/wt_$v.jsonl')])"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_dual.py tests/test_gpu_bn_adam.py > gpurun_out/r05/pytest_wt.log 2>&1; rc=$?; tail -n 2 gpurun_out/r05/pytest_wt.log; exit $rc
