"""RCCL reduce_scatter / all_reduce output-tail check on one GPU (NativeComm, world 1): every count
in a sweep must reproduce its input exactly.  Found ncclAvg (torch-bundled RCCL 2.26.6) leaving
4-16 trailing outputs unwritten; Hyperion issues "avg" as SUM + 1/world (csrc/comm/rccl_comm.cpp).

    python scripts/rccl_avg_check.py
"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

s = socket.socket()
s.bind(("127.0.0.1", 0))
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
s.close()
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from hyperion.parallel.comm import NativeComm  # noqa: E402

c = NativeComm(torch.device("cuda", 0))
bad = []
counts = [132480, 131584] + [64 * k for k in range(1, 300)] + [64 * k for k in range(2000, 2100)]
for dt in (torch.bfloat16, torch.float32):
    for op in ("avg", "sum"):
        for n in counts:
            x = torch.randn(n, device="cuda").to(dt)
            out = torch.full((n,), 7.0, device="cuda", dtype=dt)
            c.reduce_scatter(out, x, op).wait()
            torch.cuda.synchronize()
            d = (out.float() - x.float()).abs()
            if float(d.max()) > 0:
                idx = (d > 0).nonzero().flatten()
                bad.append((str(dt), op, n, int(idx.numel()), idx[:3].tolist(), idx[-3:].tolist()))
print("bad", len(bad), flush=True)
for b in bad[:40]:
    print("rs", b, flush=True)
dist.destroy_process_group()
