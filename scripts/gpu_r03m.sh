set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llama_fused.py > gpurun_out/r03m_tests.log 2>&1
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r03m_attn.jsonl 2> gpurun_out/r03m_attn.err
