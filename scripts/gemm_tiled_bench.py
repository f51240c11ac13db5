"""Tiled MFMA GEMM (gemm_tiles.hip) vs hipBLASLt (torch.matmul) on MI355X, random operands, interleaved
rounds in one process (guide §5.4 rules 24/25).

python scripts/gemm_tiled_bench.py [--sweep] [--out gpurun_out/gemm_tiled.json]
  default: square 4096/8192 NT plus the ViT-B/16 / GPT-2 / LM-256 training GEMMs (forward NT, data
  gradient NN, weight gradient TN) at the automatic plan; --sweep also times every (tile, splits)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402


def timeit(fn, iters=20, rounds=3):
    """us per call from hipGraph replays of `iters` captured calls (no host launch overhead in the
    number: the small shapes are 10-30 us, comparable to a Python-side launch)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        fn()
        with torch.cuda.graph(g, stream=s0):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s0)
    best = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g.replay()
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) * 1e3 / iters)
    return min(best)


def case(kind, M, N, K, sweep):
    C = _native.native()
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    if kind == "fwd":  # y = x wᵀ
        a, b, at, bt = r(M, K), r(N, K), False, False
        ven = lambda: torch.matmul(a, b.t())  # noqa: E731
    elif kind == "dgrad":  # dx[M, N] = dy[M, K] · W[K, N]
        a, b, at, bt = r(M, K), r(K, N), False, True
        ven = lambda: torch.matmul(a, b)  # noqa: E731
    else:  # wgrad: dW[M, N] = dy[K, M]ᵀ x[K, N]
        a, b, at, bt = r(K, M), r(K, N), True, True
        ven = lambda: torch.matmul(a.t(), b)  # noqa: E731
    ref = ven().float()
    got = C.gemm(a, b, a_tr=at, b_tr=bt).float()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    plan = C.gemm_plan(M, N, K)
    res = {"kind": kind, "M": M, "N": N, "K": K, "plan": plan, "rel_err": err}
    res["vendor_us"] = timeit(ven)
    if M <= 1024 and kind in ("fwd", "dgrad"):  # the split-K weight-streaming kernels (linear_nt / linear_nn)
        sk = (lambda: C.linear_nt(a, b)) if kind == "fwd" else (lambda: C.linear_nn(a, b))
        res["skinny_us"] = timeit(sk)
    res["hyp_us"] = timeit(lambda: C.gemm(a, b, a_tr=at, b_tr=bt))
    fl = 2.0 * M * N * K
    res["vendor_tf"] = fl / res["vendor_us"] / 1e6
    res["hyp_tf"] = fl / res["hyp_us"] / 1e6
    if sweep:
        sw = {}
        for t in (0, 1, 2):
            for s in (1, 2, 3, 4, 6, 8):
                if K // s < 256 and s > 1:
                    continue
                sw[f"t{t}s{s}"] = round(timeit(lambda: C.gemm(a, b, a_tr=at, b_tr=bt, tile=t, splits=s), iters=10,
                                               rounds=2), 1)
        res["sweep"] = sw
        res["best"] = min(sw.items(), key=lambda kv: kv[1])
    print(json.dumps(res), flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    shapes = [("fwd", 4096, 4096, 4096), ("fwd", 8192, 8192, 8192)]
    for M, D, F in [(6304, 768, 3072), (2032, 768, 3072)]:  # ViT-B/16 b32, GPT-2-small b16
        for N, K in [(3 * D, D), (D, D), (F, D), (D, F)]:
            shapes += [("fwd", M, N, K), ("dgrad", M, K, N), ("wgrad", N, K, M)]
    for N, K in [(2048, 256), (256, 2048), (768, 256)]:  # LM-256 FFN / qkv, 4064 tokens
        shapes += [("fwd", 4064, N, K), ("dgrad", 4064, K, N), ("wgrad", N, K, 4064)]
    for N, K in [(4096, 4096), (11008, 4096), (4096, 11008)]:  # Llama-2-7B projections at 128 tokens
        shapes += [("fwd", 128, N, K), ("dgrad", 128, K, N)]
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only.split(",")]
    out = [case(*s, a.sweep) for s in shapes]
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
