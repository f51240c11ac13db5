#!/bin/bash
# PMC passes over the flash-attention kernels (long causal D=128, ViT-B/16, GPT-2 shapes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmca
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P_SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"
P_RD="FETCH_SIZE,GRBM_GUI_ACTIVE"
run_pmc() {
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmca/$name" -o run -- "$@" > gpurun_out/pmca/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for pass in SQ RD; do
  eval ctr=\$P_$pass
  run_pmc long_d128_$pass "$ctr" python3 "$PWD/scripts/attn_one.py" 2 4096 16 128 1
  run_pmc vit_$pass "$ctr" python3 "$PWD/scripts/attn_one.py" 32 197 12 64 0
  run_pmc gpt2_$pass "$ctr" python3 "$PWD/scripts/attn_one.py" 8 1024 12 64 1
done
echo done
