#!/bin/bash
# round 5, call B: fused dgrad + wgrad launch — numerics, then the ResNet-50 A/B
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv_dual.py > gpurun_out/r05/pytest_dual.log 2>&1 || { tail -n 30 gpurun_out/r05/pytest_dual.log; exit 1; }
tail -n 3 gpurun_out/r05/pytest_dual.log
for v in 1 0 2 1 0 2; do
  HYPERION_CONV_DUAL=$v timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/dual_$v.jsonl 2>gpurun_out/r05/dual_$v.err || exit 1
done
for v in 1 0 2; do echo "dual=$v"; python -c "import json,sys; [print(json.loads(l)['ms_per_step']) for l in open('gpurun_out/r05/dual_$v.jsonl')]"; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_xf.py tests/test_gpu_graph_step.py > gpurun_out/r05/pytest_conv.log 2>&1
rc=$?
tail -n 3 gpurun_out/r05/pytest_conv.log
exit $rc
