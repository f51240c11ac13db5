set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_ln.py tests/test_gpu_llama_fused.py tests/test_gpu_llm_ops.py tests/test_gpu_dropout_graphs.py > gpurun_out/r03n_tests.log 2>&1 || { tail -40 gpurun_out/r03n_tests.log; exit 1; }
tail -3 gpurun_out/r03n_tests.log
timeout -k 10 300 python -u scripts/attn_bench.py > gpurun_out/r03n_attn.jsonl 2> gpurun_out/r03n_attn.err
cat gpurun_out/r03n_attn.jsonl
