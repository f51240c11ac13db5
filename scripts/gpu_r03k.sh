#!/bin/bash
# rank-r split-partial LoRA kernels + fp32 MFMA GEMM: numerics, micro-timings, C3 matmul sweep, Llama step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_llama_fused.py tests/test_gpu_gemm.py tests/test_gpu_wstream.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_k.log; grep -E "^(FAILED|E .*(assert|Error))" gpurun_out/pytest_k.log | head -8; fatal $rc
timeout -k 10 120 python3 -u scripts/lora_bench.py 2>/dev/null; fatal $?
timeout -k 10 300 python3 -u -c "
import json, sys
sys.path.insert(0, '.')
from hyperion.bench.hardware import matmul_tflops
rows = []
for p in ('bf16', 'fp16', 'fp32'):
    for n in (1024, 2048, 4096, 8192):
        for k in ('hyperion', 'torch'):
            r = matmul_tflops(n, p, k, 'proper'); rows.append(r)
            print(p, n, k, round(r['TFLOPS'], 1), r.get('Tile'), flush=True)
json.dump(rows, open('gpurun_out/c3_matmul.json', 'w'), indent=1)
" 2>&1 | grep -v amdgpu; fatal $?
timeout -k 10 300 python3 -u scripts/run_model_step.py llamagraph20 > gpurun_out/llama_fused.json 2> gpurun_out/llama_fused.err; rc=$?; echo "llama fused rc=$rc"; tail -1 gpurun_out/llama_fused.json | cut -c1-200; fatal $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; echo "trace llama rc=$?"
