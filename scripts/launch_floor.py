"""Per-kernel cost inside a hipGraph on MI355X: N back-to-back launches of (a) an 8-element fill,
(b) the BN finalize over 784 x 64 partials, (c) the same finalize after a 51 MB producer write.
Prints us per kernel (graph replay wall time / N)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C_ = _native.native()
dev = torch.device("cuda")


def graph_time(fn, n=100, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


small = torch.zeros(8, device=dev)
print("fill8          us/kernel", round(graph_time(lambda: small.fill_(1.0)), 2))
x = torch.randn(32, 64, 56, 56, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 64, 1, 1, device=dev) * 0.1).bfloat16().contiguous(memory_format=torch.channels_last)
sums = torch.zeros(8, 2, w.shape[0], device="cuda", dtype=torch.float64)
y, psum, psq = C_.conv_fwd(x, w, 1, 1, 0, 0, True, sums=sums)
bw, bb = torch.ones(64, device=dev), torch.zeros(64, device=dev)
rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
print("sums", tuple(sums.shape))
print("conv1x1+stats   us/kernel", round(graph_time(lambda: C_.conv_fwd(x, w, 1, 1, 0, 0, True), n=20), 2))
print("bn_fwd_sums us/call      ", round(graph_time(lambda: C_.bn_fwd_sums(y, None, sums, bw, bb, rm, rv, 0.1, 1e-5, True), n=50), 2))
big = torch.empty(51 * 2**20 // 4, device=dev)
print("fill51MB        us/kernel", round(graph_time(lambda: big.fill_(1.0), n=20), 2))
print("fill51MB+fill8  us/pair  ", round(graph_time(lambda: (big.fill_(1.0), small.fill_(2.0)), n=20), 2))
