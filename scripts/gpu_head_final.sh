# Fused classifier head + MSE as the bench default: tests, smoke, bench (default / torch loss / DDP world 1), step trace
set -o pipefail
mkdir -p gpurun_out/hf
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_linear_mse.py tests/test_gpu_ddp_graph.py > gpurun_out/hf/test.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/hf/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/hf/bench_default.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/hf/bench_head.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --loss torch > gpurun_out/hf/bench_torch.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/hf/bench_head2.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --loss torch > gpurun_out/hf/bench_torch2.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --ddp-world1 1 > gpurun_out/hf/bench_ddp1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hf/prof -o run -- python bench.py --steps 10 --warmup 5 > gpurun_out/hf/prof.log 2>&1
echo rc=$?
tail -2 gpurun_out/hf/test.log; tail -1 gpurun_out/hf/smoke.log | cut -c1-200; for f in gpurun_out/hf/bench_*.log; do echo $f; grep ms_per_step $f | cut -c1-160; done
