#!/bin/bash
# round 5: fp32 eager linears on the vendor ops — transformer GPU tests, CustomTransformer fp32 host
# profile (plain vs the fused Functions), baseline model rows
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py tests/test_gpu_llm_ops.py tests/test_gpu_attn_ln.py tests/test_gpu_graph_step.py tests/test_gpu_dropout_graphs.py tests/test_gpu_round4.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1; do
  HYPERION_FP32_FUSED=$v timeout -k 10 300 python scripts/eager_host_prof.py ct32 > $O/ct32_fused$v.log 2>&1 || { tail -5 $O/ct32_fused$v.log; exit 1; }
  grep "^{" $O/ct32_fused$v.log
done
timeout -k 10 900 python -u -m hyperion.cli.bench_models --only baseline --out $O/models > $O/models.log 2>&1 || { tail -20 $O/models.log; exit 1; }
cat $O/models/*fp32*.csv
