#!/bin/bash
# Transformer side: dropout-fusion tests, LM-256 / GPT-2-small graphed steps, GPT-2 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-lm}
mkdir -p gpurun_out/r04/$tag
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_round4.py tests/test_gpu_attn_ln.py tests/test_gpu_gemm_tiled.py tests/test_gpu_dropout_graphs.py > gpurun_out/r04/$tag/pytest.log 2>&1
rc=$?
echo tests rc=$rc
tail -3 gpurun_out/r04/$tag/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/run_model_step.py lmgraph > gpurun_out/r04/$tag/lm256.json 2>gpurun_out/r04/$tag/lm256.err && \
timeout -k 10 300 python -u scripts/run_model_step.py gpt2 > gpurun_out/r04/$tag/gpt2.json 2>gpurun_out/r04/$tag/gpt2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/r04/$tag/prof" -o run -- python3 scripts/run_model_step.py gpt2 > /dev/null 2>&1 && \
python3 scripts/kstats.py $(ls gpurun_out/r04/$tag/prof/run_kernel_trace.csv gpurun_out/r04/$tag/prof/*/run_kernel_trace.csv 2>/dev/null | head -1) 40 0.5 > gpurun_out/r04/$tag/gpt2_kstats.txt
echo rc=$?
cut -c1-400 gpurun_out/r04/$tag/lm256.json gpurun_out/r04/$tag/gpt2.json; grep -c dropout_k gpurun_out/r04/$tag/gpt2_kstats.txt || true; head -20 gpurun_out/r04/$tag/gpt2_kstats.txt
