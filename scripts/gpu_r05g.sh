#!/bin/bash
# round 5, call G: write-through stores (hazard fix) + persistent convs — tests, then bench A/B
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_persist.py > gpurun_out/r05/pytest_persist.log 2>&1; rc=$?
tail -n 15 gpurun_out/r05/pytest_persist.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_dual.py tests/test_gpu_bn_adam.py tests/test_gpu_conv_xf.py tests/test_gpu_pool.py tests/test_gpu_graph_step.py tests/test_gpu_llama_fused.py tests/test_gpu_linear.py tests/test_gpu_llm_ops.py > gpurun_out/r05/pytest_wt2.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r05/pytest_wt2.log | head; tail -n 3 gpurun_out/r05/pytest_wt2.log; exit 1; }
tail -n 2 gpurun_out/r05/pytest_wt2.log
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/g_plain.jsonl 2>>gpurun_out/r05/g.err || exit 1
  [ $rc -eq 0 ] || continue
  HYPERION_CONV_PERSIST=1 timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> gpurun_out/r05/g_persist.jsonl 2>>gpurun_out/r05/g.err || exit 1
done
for f in gpurun_out/r05/g_plain.jsonl gpurun_out/r05/g_persist.jsonl; do [ -f $f ] && python -c "import json,sys; print(sys.argv[1], [json.loads(l)['ms_per_step'] for l in open(sys.argv[1])])" $f; done
exit 0
