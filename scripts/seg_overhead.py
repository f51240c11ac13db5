"""GPU cost of segmented-graph boundaries (train/segments.py): a fixed chain of matmul kernels
captured as ONE graph vs split into K segments at no-op holes, and at holes that fork / join a
side stream with events (the shape of a DDP all-reduce issue / wait).  One JSON line per case."""
import json
import sys

import torch

sys.path.insert(0, ".")
from hyperion.train.segments import SegmentedGraph, eager  # noqa: E402

a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
side = torch.cuda.Stream()
KERNELS = 240


def body(k_holes, fork):
    x = a
    every = KERNELS // (k_holes + 1) if k_holes else KERNELS + 1
    for i in range(KERNELS):
        x = torch.mm(x, a) * 0.01
        if k_holes and (i + 1) % every == 0 and (i + 1) // every <= k_holes:
            if fork:
                def act():
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        torch.cuda._sleep(10)
                    torch.cuda.current_stream().wait_stream(side)
                eager(act)
            else:
                eager(lambda: None)
    return x


body(0, False)  # eager warm-up: vendor GEMM handles exist before any capture
torch.cuda.synchronize()
for k_holes, fork in ((0, False), (1, False), (3, False), (10, False), (3, True), (10, True)):
    seg = SegmentedGraph()
    seg.capture(lambda: body(k_holes, fork))
    for _ in range(3):
        seg.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        seg.replay()
    e.record()
    e.synchronize()
    print(json.dumps({"holes": k_holes, "fork_join": fork, "segments": seg.num_segments,
                      "ms_per_replay": round(s.elapsed_time(e) / 20, 4)}), flush=True)
