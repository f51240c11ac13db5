#!/bin/bash
# attention tests + micro bench, then kernel traces of the graphed Llama-2-7B LoRA and ViT-B/16 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llama_fused.py > gpurun_out/r03o_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03o_tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/r03o_tests.log; exit $rc; }
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r03o_attn.jsonl 2> gpurun_out/r03o_attn.err; rc=$?; cat gpurun_out/r03o_attn.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_llama" -o run -- python3 "$PWD/scripts/run_model_step.py" llamagraph > gpurun_out/trace_llama.log 2>&1; rc=$?; echo "trace llama rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace_vit" -o run -- python3 "$PWD/scripts/run_model_step.py" vitgraph > gpurun_out/trace_vit.log 2>&1; rc=$?; echo "trace vit rc=$rc"; [ $rc -ne 0 ] && exit $rc

timeout -k 10 300 python3 -u scripts/eager_host_prof.py vit > gpurun_out/r03o_vit_eager_prof.txt 2>&1; echo "host prof rc=$?"
