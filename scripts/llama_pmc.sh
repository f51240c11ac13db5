#!/bin/bash
# Llama-2-7B LoRA step: what caps the weight-streaming GEMM (ws_gemm_k)?  One eager step per counter
# pass (no tracing in the same run), a kernel trace for the timings, the table built on the box and
# the raw files compressed.
#   bash scripts/llama_pmc.sh [outdir]
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=${1:-gpurun_out/suite/llama_pmc}; mkdir -p $O
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VMEM_RD,SQ_WAVES,SQ_INST_LEVEL_VMEM,GRBM_GUI_ACTIVE"
P2="TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_DRAM_sum,GRBM_GUI_ACTIVE"
P3="TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_STALL_MULTI_MISS_sum,TCP_UTCL1_THRASHING_STALL_sum,GRBM_GUI_ACTIVE"
P4="TCP_TCC_READ_REQ_sum,TCP_TCC_READ_REQ_LATENCY_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TCR_TCP_STALL_CYCLES_sum,GRBM_GUI_ACTIVE"
P5="TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum,TCC_TAG_STALL_sum,GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  rm -rf "$O/raw"
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$PWD/$O/raw" -o run -- \
    python3 scripts/run_model_step.py llama1 > "$O/pass_$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/pass_$i.log"; exit 1; }
  f=$(find "$O/raw" -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] || { echo "pass $i: no counter file"; find "$O/raw" | head; exit 1; }
  cp "$f" "$O/llama_P$i.csv" && rm -rf "$O/raw"
  echo "pass $i ok"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/kt" -o run -- \
  python3 scripts/run_model_step.py llama1 > "$O/kt.log" 2>&1 || { echo "trace failed"; tail -5 "$O/kt.log"; exit 1; }
f=$(find "$O/kt" -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && cp "$f" "$O/kernel_trace.csv"
f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$O/kernel_stats.csv"
rm -rf "$O/kt"
python3 scripts/ws_pmc_table.py $O > $O/ws_pmc_table.md && head -20 $O/ws_pmc_table.md
gzip -f $O/llama_P*.csv $O/kernel_trace.csv
