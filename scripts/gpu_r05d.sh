#!/bin/bash
# round 5, call D: BN dx + weight-gradient fusion — numerics, ResNet-50 A/B (bn | dgrad | separate)
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv_dual.py > gpurun_out/r05/pytest_dual2.log 2>&1 || { tail -n 40 gpurun_out/r05/pytest_dual2.log; exit 1; }
tail -n 2 gpurun_out/r05/pytest_dual2.log
for i in 1 2; do
  for v in bn dgrad 0; do
    HYPERION_WGRAD_FUSE=$v timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/fuse_$v.jsonl 2>gpurun_out/r05/fuse_$v.err || exit 1
  done
done
for v in bn dgrad 0; do echo "fuse=$v"; python -c "import json,sys; print([json.loads(l)['ms_per_step'] for l in open('gpurun_out/r05/fuse_$v.jsonl')])"; done
bash scripts/gpu_r05_trace.sh fusebn > /dev/null 2>&1; grep "step -2" -A 12 gpurun_out/r05/fusebn_step.txt
