"""Per-kernel floor of back-to-back dependent kernels on one stream: eager vs hipGraph replay, tiny
vs 1 MB elementwise kernels (run under different HIP env knobs by the caller)."""
import json
import os
import sys

import torch


def per_kernel_us(n_elem, graph, n=400, reps=5):
    x = torch.zeros(n_elem, device="cuda")

    def body():
        for _ in range(n):
            x.add_(1.0)

    body()
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            body()
        run = g.replay
    else:
        run = body
    run()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return best


tag = sys.argv[1] if len(sys.argv) > 1 else "default"
res = {"tag": tag, "env": {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_", "HIP_", "GPU_", "ROC_", "AMD_"))}}
for n_elem in (1, 1 << 18):
    for graph in (False, True):
        res[f"{'graph' if graph else 'eager'}_{n_elem}"] = round(per_kernel_us(n_elem, graph), 2)
print(json.dumps(res), flush=True)
