"""Transformer GEMM shapes: Hyperion's MFMA implicit-GEMM kernel (conv_igemm.hip as linear_nt /
linear_nn, conv_wgrad.hip at 1x1 for dW) vs the vendor GEMM (F.linear / torch.mm -> hipBLASLt),
in-graph per-launch us.  Output: gpurun_out/gemm_shapes.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C_ = _native.native()


def gtime(fn, n=10, reps=5):
    import time
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


def main():
    rows = []
    # (M, K, N): y[M,N] = x[M,K] w[N,K]^T  — ViT-B/16 b32, GPT-2-small b16x127, LM-256 b32x127
    for M, K, N in [(6304, 768, 2304), (6304, 768, 768), (6304, 768, 3072), (6304, 3072, 768),
                    (2032, 768, 2304), (2032, 768, 3072), (2032, 3072, 768), (4064, 256, 2048), (4064, 2048, 256),
                    (8192, 8192, 8192)]:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        dy = torch.randn(M, N, device="cuda").bfloat16()
        fl = 2.0 * M * N * K
        r = {"M": M, "K": K, "N": N}
        r["fwd_vendor"] = gtime(lambda: torch.nn.functional.linear(x, w))
        for bn in (64, 128):
            r[f"fwd_hyp_bn{bn}_s1"] = gtime(lambda: C_.linear_nt(x, w, splits=1, bn=bn))
        r["dgrad_vendor"] = gtime(lambda: dy @ w)
        for bn in (64, 128):
            r[f"dgrad_hyp_bn{bn}_s1"] = gtime(lambda: C_.linear_nn(dy, w, splits=1, bn=bn))
        r["wgrad_vendor"] = gtime(lambda: dy.t() @ x)
        r["wgrad_hyp"] = gtime(lambda: C_.conv_wgrad(dy.view(M, N, 1, 1), x.view(M, K, 1, 1), 1, 1, 1, 1, 0, 0))
        for k in list(r):
            if k not in ("M", "K", "N"):
                r[k.replace("_", "_TF_", 1) if False else k] = round(r[k], 1)
        r["tflops_vendor_fwd"] = round(fl / r["fwd_vendor"] / 1e6, 0)
        print(json.dumps(r), flush=True)
        rows.append(r)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(rows, open("gpurun_out/gemm_shapes.json", "w"), indent=1)


if __name__ == "__main__":
    main()
