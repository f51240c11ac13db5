#!/bin/bash
# Round-2 GPU call I: smoke, full GPU suite (tiled GEMM + debug build included), headline bench,
# PMC passes on the tiled GEMM (8192^3 and the ViT fc1 weight gradient) next to the 128^2 baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log | cut -c1-200; fatal $rc
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --json-out gpurun_out/bench_graph.json > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; fatal $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; fatal $rc
P_SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"
P_RD="FETCH_SIZE,GRBM_GUI_ACTIVE"
P_WR="WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"
for pass in SQ RD WR; do
  eval ctr=\$P_$pass
  for tgt in gemm gemm_tiled gemm_tiled_wgrad; do
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmc2/${tgt}_$pass" -o run -- python3 "$PWD/scripts/hw_one.py" $tgt > gpurun_out/pmc2/${tgt}_$pass.log 2>&1
    rc=$?; echo "pmc ${tgt}_$pass rc=$rc $(grep '^{' gpurun_out/pmc2/${tgt}_$pass.log)"; fatal $rc
  done
done
echo done
