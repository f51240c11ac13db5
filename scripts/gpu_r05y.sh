#!/bin/bash
# round 5, call Y: BN apply / dx kernels issue their first rows' loads before the inline finalize —
# numerics tests, bench x3, step trace (per-kernel times vs profiles/r05/trace_resnet50_step_4.42ms.txt)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bn_adam.py tests/test_gpu_conv_dual.py tests/test_gpu_round4.py tests/test_gpu_graph_step.py tests/test_gpu_conv.py > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do timeout -k 10 150 python bench.py --steps 50 --warmup 10 >> $O/bench.jsonl 2>>$O/err || exit 1; done
python -c "import json; print([json.loads(l)['ms_per_step'] for l in open('$O/bench.jsonl')])"
bash scripts/gpu_r05_trace.sh step_r05y > /dev/null || exit 1
grep -E "busy|bn_apply_k|bn_bwd_dx_k" gpurun_out/r05/step_r05y_step.txt | tail -8
