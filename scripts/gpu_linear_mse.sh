set -o pipefail
mkdir -p gpurun_out/lm
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_linear_mse.py > gpurun_out/lm/test.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --loss head > gpurun_out/lm/bench_head.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/lm/bench_torch.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --loss head > gpurun_out/lm/bench_head2.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/lm/bench_torch2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lm/prof -o run -- python bench.py --steps 10 --warmup 5 --loss head > gpurun_out/lm/prof.log 2>&1
echo rc=$?
tail -3 gpurun_out/lm/test.log; grep -h ms_per_step gpurun_out/lm/bench_*.log | cut -c1-200
python3 -c "
import sqlite3
c=sqlite3.connect('gpurun_out/lm/prof/run_results.db')
for r in c.execute(\"select name, count(*), avg(end-start)/1000.0 from kernels where name like '%linear_mse%' or name like '%gap_%' group by name\"): print(r[1], round(r[2],2), r[0][:70])
"
