#!/bin/bash
# PMC passes over single GEMM shapes: native ping-pong / classic tiles vs the vendor GEMM.
#   bash scripts/gemm_pmc.sh [outdir]   (one rocprofv3 run per counter pass; summary on the box)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=${1:-gpurun_out/suite/gemm_pmc}; mkdir -p $O
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_SALU,SQ_INSTS_VALU,GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"
P4="FETCH_SIZE,GRBM_GUI_ACTIVE"
IFS=';' read -ra CFGS <<< "${GEMM_PMC_CFGS:-8192 8192 8192 8 1;8192 8192 8192 0 1;8192 8192 8192 0 1 vendor;6304 2304 768 8 1;6304 2304 768 0 1 vendor;6304 768 3072 10 1;6304 768 3072 0 1 vendor}"
for cfg in "${CFGS[@]}"; do
  tag=$(echo $cfg | tr ' ' '-')
  i=0
  for pass in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    rm -rf "$O/raw"
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$PWD/$O/raw" -o run -- \
      python3 scripts/micro/gemm_one.py $cfg > "$O/$tag.P$i.log" 2>&1 || { echo "$tag pass $i failed"; tail -3 "$O/$tag.P$i.log"; exit 1; }
    f=$(find "$O/raw" -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] || { echo "$tag pass $i: no counter file"; find "$O/raw" | head; exit 1; }
    mkdir -p "$O/${tag}_P$i" && cp "$f" "$O/${tag}_P$i/run_counter_collection.csv"
  done
  rm -rf "$O/raw"
  echo "$tag ok"
done
python3 scripts/pmc_summary.py $O --out $O/gemm_pmc_table.md | cut -c1-260
