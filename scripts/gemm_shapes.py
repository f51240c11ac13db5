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


def skinny():
    """Llama-2-7B LoRA step shapes (batch 1 x 128 tokens): weight-streaming GEMMs.  Four weight
    copies are cycled inside the graph so each launch reads its weight from HBM (4 x 86 MB > the
    256 MB Infinity Cache), as in the real step."""
    rows = []
    M = 128
    for K, N in [(4096, 4096), (4096, 11008), (11008, 4096)]:
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(4)]
        x = torch.randn(M, K, device="cuda").bfloat16()
        dy = torch.randn(M, N, device="cuda").bfloat16()
        U = torch.randn(M, 16, device="cuda").bfloat16()
        V = torch.randn(16, N, device="cuda").bfloat16()
        it = {"i": 0}

        def nxt():
            it["i"] = (it["i"] + 1) % 4
            return ws[it["i"]]

        r = {"M": M, "K": K, "N": N, "floor_us": round(N * K * 2 / 6.0e6, 1)}
        r["fwd_vendor"] = gtime(lambda: torch.nn.functional.linear(x, nxt()), n=8)
        r["fwd_hyp"] = gtime(lambda: C_.linear_nt(x, nxt()), n=8)
        r["fwd_hyp_lora"] = gtime(lambda: C_.linear_nt(x, nxt(), U=U, V=V), n=8)
        r["fwd_vendor_lora"] = gtime(lambda: torch.addmm(torch.nn.functional.linear(x, nxt()), U, V), n=8)
        r["dgrad_vendor"] = gtime(lambda: dy @ nxt(), n=8)
        r["dgrad_hyp"] = gtime(lambda: C_.linear_nn(dy, nxt()), n=8)
        for nb in (2, 3, 4):
            C_.conv_set_stages(nb, 0)
            for sp in (2, 4, 8, 16):
                r[f"fwd_hyp_s{sp}_nb{nb}"] = gtime(lambda: C_.linear_nt(x, nxt(), splits=sp), n=8)
                r[f"dgrad_hyp_s{sp}_nb{nb}"] = gtime(lambda: C_.linear_nn(dy, nxt(), splits=sp), n=8)
            for bn in (64, 128):
                r[f"fwd_hyp_bn{bn}_nb{nb}"] = gtime(lambda: C_.linear_nt(x, nxt(), bn=bn), n=8)
        C_.conv_set_stages(0, 0)
        r = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        print(json.dumps(r), flush=True)
        rows.append(r)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(rows, open("gpurun_out/gemm_skinny.json", "w"), indent=1)


if __name__ == "__main__":
    if "--skinny" in sys.argv:
        skinny()
    else:
        main()
