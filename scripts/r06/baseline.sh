#!/bin/bash
# round-6 baseline on a fresh box: bench.py (driver contract) + native-vs-vendor GEMM sweep
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06/baseline; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python scripts/micro/gemm_sweep.py 8192 8192 8192 6304 2304 768 6304 768 768 6304 3072 768 6304 768 3072 2048 2304 768 2048 768 3072 > $O/gemm_sweep.jsonl 2> $O/gemm_sweep.err || { tail -5 $O/gemm_sweep.err; exit 1; }
cut -c1-400 $O/gemm_sweep.jsonl
