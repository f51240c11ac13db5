#!/bin/bash
# PMC counters (one pass each, own run) for the conv kernels on a layer3 3x3 and a layer1 1x1 shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_MFMA,SQ_WAVES,SQ_INST_LEVEL_VMEM,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum,GRBM_GUI_ACTIVE"
i=0
for shape in "32 256 14 256 3 1 1" "32 64 56 256 1 1 0"; do
  for pass in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$PWD/gpurun_out/pmc/p$i" -o run -- python3 "$PWD/scripts/conv_one.py" $shape > gpurun_out/pmc_$i.log 2>&1
    echo "pass $i rc=$?"
  done
done
