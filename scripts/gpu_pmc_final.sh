#!/bin/bash
# PMC roofline refresh (one rocprofv3 run per counter pass): tiled GEMM 8192^3, 128^2 baseline GEMM,
# STREAM add 500M, ResNet-50 conv shapes (layer1 3x3 / 1x1, layer3 3x3) fwd + dgrad + wgrad
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcf
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P_SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"
P_RD="FETCH_SIZE,GRBM_GUI_ACTIVE"
P_WR="WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"
run_pmc() {
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmcf/$name" -o run -- "$@" > gpurun_out/pmcf/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for pass in SQ RD WR; do
  eval ctr=\$P_$pass
  run_pmc gemm_tiled_$pass "$ctr" python3 "$PWD/scripts/hw_one.py" gemm_tiled
  run_pmc gemm_tiled_wgrad_$pass "$ctr" python3 "$PWD/scripts/hw_one.py" gemm_tiled_wgrad
  run_pmc stream_$pass "$ctr" python3 "$PWD/scripts/hw_one.py" stream
  run_pmc conv_l1_3x3_$pass "$ctr" python3 "$PWD/scripts/conv_one.py" 32 64 56 64 3 1 1
  run_pmc conv_l3_3x3_$pass "$ctr" python3 "$PWD/scripts/conv_one.py" 32 256 14 256 3 1 1
  run_pmc conv_l1_1x1_$pass "$ctr" python3 "$PWD/scripts/conv_one.py" 32 64 56 256 1 1 0
done
echo done
