#!/bin/bash
# round 5: no-grad direct forward dispatch (fused inference host overhead) — op tests + fusion bench
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_attn_ln.py tests/test_gpu_linear.py tests/test_gpu_llm_ops.py tests/test_gpu_embedding.py tests/test_gpu_pool.py tests/test_gpu_round4.py tests/test_gpu_llama_fused.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for dt in bf16 fp32; do
  timeout -k 10 300 python -m hyperion.cli.fusion_bench --base_dir $O/$dt --dtype $dt --repeat 200 > $O/fusion_$dt.log 2>&1 || { tail -10 $O/fusion_$dt.log; exit 1; }
  grep -v amdgpu $O/fusion_$dt.log
done
