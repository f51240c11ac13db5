#!/bin/bash
# RCCL through Hyperion's native communicator with two ranks on the one GPU (duplicate-device probe)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
HYPERION_SAME_DEVICE=1 timeout -k 10 120 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 -m hyperion.cli.test_rccl --backend native > gpurun_out/rccl_2rank_1gpu.log 2>&1
echo "rccl 2-rank same-GPU rc=$?"; tail -12 gpurun_out/rccl_2rank_1gpu.log | cut -c1-300
timeout -k 10 200 python3 -c "
import sys, json; sys.path.insert(0, '.')
from hyperion.bench.models import bench_lm_step
print(json.dumps(bench_lm_step(precision='bf16', graph=False, model='gpt2_small', batch=16)))
" > gpurun_out/gpt2_eager.log 2>&1; echo "gpt2 eager rc=$?"; grep '^{' gpurun_out/gpt2_eager.log | cut -c1-200
