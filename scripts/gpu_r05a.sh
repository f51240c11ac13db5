#!/bin/bash
# round 5, call A: ResNet-50 wgrad-overlap A/B + the update-parity / comm tests
set -o pipefail
mkdir -p gpurun_out/r05
for v in base side nowgrad base side nowgrad; do
  timeout -k 10 150 python scripts/resnet_variants.py $v --steps 50 --warmup 10 >> gpurun_out/r05/var_$v.jsonl 2>gpurun_out/r05/var_$v.err || exit 1
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_fsdp_graph.py tests/test_gpu_ddp_segments.py tests/test_gpu_ddp_graph.py > gpurun_out/r05/pytest_a.log 2>&1
rc=$?
tail -n 3 gpurun_out/r05/var_*.jsonl
tail -n 5 gpurun_out/r05/pytest_a.log
exit $rc
