#!/bin/bash
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05gs; mkdir -p $O
timeout -k 10 300 python scripts/micro/gemm_sweep.py 2048 50257 768 6304 3072 768 6304 768 3072 2048 3072 768 2048 2304 768 8192 8192 8192 > $O/sweep.jsonl 2>&1 || { tail -5 $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl
