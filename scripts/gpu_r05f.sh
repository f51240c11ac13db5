#!/bin/bash
# round 5, call F: write-through stores with the hazard fix — broad GPU tests + bench
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_dual.py tests/test_gpu_bn_adam.py tests/test_gpu_conv_xf.py tests/test_gpu_pool.py tests/test_gpu_graph_step.py tests/test_gpu_llama_fused.py tests/test_gpu_linear.py tests/test_gpu_llm_ops.py > gpurun_out/r05/pytest_wt2.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r05/pytest_wt2.log | head; tail -n 3 gpurun_out/r05/pytest_wt2.log; exit 1; }
tail -n 2 gpurun_out/r05/pytest_wt2.log
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/wt2_sc1.jsonl 2>>gpurun_out/r05/wt.err || exit 1
done
python -c "import json,sys; print([json.loads(l)['ms_per_step'] for l in open('gpurun_out/r05/wt2_sc1.jsonl')])"
