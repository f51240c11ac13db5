#!/bin/bash
# Round-2 GPU call B: per-layer conv timings, PMC counter passes (one run per pass) on the top conv
# shapes + the MFMA GEMM 8192^3 + STREAM add 500M, STREAM launch-mode sweep, RCCL 2 ranks on 1 GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -c "
import json, sys; sys.path.insert(0, '.')
from hyperion.bench.conv_shapes import run
rows = run(32, sweep=False)
json.dump(rows, open('gpurun_out/conv_shapes.json', 'w'), indent=1)
" > gpurun_out/conv_shapes.log 2>&1; rc=$?; echo "shapes rc=$rc"; fatal $rc
timeout -k 10 120 python3 scripts/hw_one.py sweep > gpurun_out/stream_sweep.log 2>&1; rc=$?; echo "sweep rc=$rc"; fatal $rc
P_SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"
P_RD="FETCH_SIZE,GRBM_GUI_ACTIVE"
P_WR="WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"
i=0
run_pmc() {  # name counters cmd...
  local name=$1 ctr=$2; shift 2
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmc/$name" -o run -- "$@" > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; fatal $rc
}
for pass in SQ RD WR; do
  eval ctr=\$P_$pass
  run_pmc gemm_$pass "$ctr" python3 "$PWD/scripts/hw_one.py" gemm
  run_pmc stream_$pass "$ctr" python3 "$PWD/scripts/hw_one.py" stream
  run_pmc conv_l1_3x3_$pass "$ctr" python3 "$PWD/scripts/conv_one.py" 32 64 56 64 3 1 1
  run_pmc conv_l3_3x3_$pass "$ctr" python3 "$PWD/scripts/conv_one.py" 32 256 14 256 3 1 1
  run_pmc conv_l1_1x1_$pass "$ctr" python3 "$PWD/scripts/conv_one.py" 32 64 56 256 1 1 0
done
# RCCL: two ranks on the one GPU through Hyperion's communicator (duplicate-GPU support probe)
HYPERION_SAME_DEVICE=1 timeout -k 10 90 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 -m hyperion.cli.test_rccl --backend native > gpurun_out/rccl_2rank_1gpu.log 2>&1
echo "rccl 2-rank same-GPU rc=$?"; tail -5 gpurun_out/rccl_2rank_1gpu.log | cut -c1-300
timeout -k 10 90 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29612 -m hyperion.cli.test_rccl --backend native --sweep --out gpurun_out/rccl_sweep_w1.json > gpurun_out/rccl_w1.log 2>&1
echo "rccl w1 rc=$?"; tail -3 gpurun_out/rccl_w1.log | cut -c1-300
echo done
