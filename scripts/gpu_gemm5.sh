#!/bin/bash
# tiled GEMM after the b128 lane-group swizzle fix: numerics, PMC (SQ pass), shape bench, transformer steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm_tiled.py tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
P_SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P_SQ --output-format csv -d "$PWD/gpurun_out/pmc3/gemm_tiled_SQ" -o run -- python3 "$PWD/scripts/hw_one.py" gemm_tiled > gpurun_out/pmc3/gemm_tiled_SQ.log 2>&1; rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/gemm_tiled_bench.py --sweep --out gpurun_out/gemm_tiled.json > gpurun_out/gemm_tiled.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_gemm3.sh
