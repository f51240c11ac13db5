"""Where does a small conv launch's time go?  In-graph per-launch times of the same 1x1 GEMM shape
through: conv_fwd with / without the BN-stats epilogue, each tile, and the plain MFMA GEMM kernel
(gemm_nt) on the identical [M, K] x [K, N]; plus hipBLASLt (torch.matmul)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C_ = _native.native()


def gtime(fn, n=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
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


for (N, C, H, K) in [(32, 256, 14, 1024), (32, 1024, 14, 256), (32, 64, 56, 256), (32, 512, 28, 128), (32, 128, 28, 512)]:
    x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 1, 1, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    M = N * H * H
    a = x.permute(0, 2, 3, 1).reshape(M, C)
    b = w.reshape(K, C)
    out = {"shape": (N, C, H, K), "M": M}
    for bm, bn in ((64, 64), (128, 64), (128, 128)):
        out[f"conv_{bm}x{bn}_stats"] = round(gtime(lambda: C_.conv_fwd(x, w, 1, 1, 0, 0, True, bm, bn, 1)), 1)
        out[f"conv_{bm}x{bn}_nostats"] = round(gtime(lambda: C_.conv_fwd(x, w, 1, 1, 0, 0, False, bm, bn, 1)), 1)
    if M % 128 == 0 and K % 128 == 0:
        out["gemm_nt"] = round(gtime(lambda: C_.gemm_nt(a, b, None, 1.0, 64)), 1)
    out["hipblaslt"] = round(gtime(lambda: torch.matmul(a, b.t())), 1)
    out["copy_out_bytes_us"] = round(gtime(lambda: torch.empty(M, K, device="cuda", dtype=torch.bfloat16).fill_(1.0)), 1)
    print(out, flush=True)
