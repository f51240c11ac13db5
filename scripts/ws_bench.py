"""Weight-streaming GEMM vs the round-2 split-K kernel vs hipBLASLt on the Llama-2-7B LoRA shapes.

Cold-weight timing: each timed call reads a different weight tensor from a pool larger than the
256 MiB Infinity Cache, so the effective bandwidth is the HBM stream the training step sees.
Writes gpurun_out/ws_bench.json.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C = _native.native()
dev = "cuda"


def timed(fn, pool, reps=3):
    """median device time (us) of one call, cycling cold weights from `pool`"""
    for w in pool[:2]:
        fn(w)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1_000_000)
        s.record()
        for w in pool:
            fn(w)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / len(pool))
    return statistics.median(ts)


def pool_of(shape, nbytes_min=640 << 20):
    n = max(3, -(-nbytes_min // (shape[0] * shape[1] * 2)))
    return [(torch.randn(*shape, device=dev) * 0.02).bfloat16() for _ in range(n)]


M = int(os.environ.get("WS_M", "128"))
SLAB16 = os.environ.get("HYPERION_WS_SLAB", "bf16") != "fp32"  # the Llama layer's slab dtype
shapes = [  # (name, N out, K in) of y = x Wᵀ; dgrad rows use W [N, K] read as NN
    ("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
]
out = []
for name, N, K in shapes:
    pool = pool_of((N, K))
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    wb = N * K * 2
    r = {"name": name, "M": M, "N": N, "K": K, "weight_MB": wb / 1e6}
    r["ws_nt"] = timed(lambda w: C.ws_linear(x, w), pool)
    r["ws_nn"] = timed(lambda w: C.ws_linear(dy, w, nn=True), pool)
    r["ws_nt_gemm_only"] = timed(lambda w: C.ws_gemm_part(x, w, slab16=SLAB16), pool)
    r["ws_nn_gemm_only"] = timed(lambda w: C.ws_gemm_part(dy, w, nn=True, slab16=SLAB16), pool)
    # M split in two 64-row blocks with twice the slice length: half the slab bytes
    r["ws_nt_mf4"] = timed(lambda w: C.ws_linear(x, w, mf=4, kr=1024, G=max(1, 256 // (2 * -(-K // 1024)))), pool)
    r["ws_nn_mf4"] = timed(lambda w: C.ws_linear(dy, w, nn=True, mf=4, kr=1024, G=max(1, 256 // (2 * -(-N // 1024)))), pool)
    if N <= 12288:
        r["r02_linear_nt"] = timed(lambda w: C.linear_nt(x, w), pool)
        r["r02_linear_nn"] = timed(lambda w: C.linear_nn(dy, w), pool)
    r["hipblaslt_nt"] = timed(lambda w: torch.nn.functional.linear(x, w), pool)
    r["hipblaslt_nn"] = timed(lambda w: dy @ w, pool)
    plan_nt = C.ws_plan(M, N, K, False)
    plan_nn = C.ws_plan(M, K, N, True)
    r["plan_nt"], r["plan_nn"] = plan_nt, plan_nn
    # sweep: m-block rows (mf), slice length, column groups, fragments per chunk
    sweep = {}
    for mf, krs in ((8, (256, 384, 512)), (4, (512, 1024)), (2, (1024, 2048))):
        MB = -(-M // (16 * mf))
        for kr in krs:
            S = -(-K // kr)
            for G in sorted({max(1, 256 // (S * MB)), max(1, 512 // (S * MB))}):
                for nf in (1, 2, 4):
                    k = f"nt_mf{mf}_kr{kr}_G{G}_nf{nf}"
                    try:
                        sweep[k] = timed(lambda w: C.ws_gemm_part(x, w, mf=mf, kr=kr, G=G, nf=nf, slab16=SLAB16), pool, 2)
                    except RuntimeError as ex:  # unsupported plan
                        sweep[k] = str(ex)[:60]
            S = -(-N // kr)
            for G in sorted({max(1, 256 // (S * MB)), max(1, 512 // (S * MB))}):
                k = f"nn_mf{mf}_kr{kr}_G{G}"
                try:
                    sweep[k] = timed(lambda w: C.ws_gemm_part(dy, w, nn=True, mf=mf, kr=kr, G=G, slab16=SLAB16), pool, 2)
                except RuntimeError as ex:
                    sweep[k] = str(ex)[:60]
    r["sweep"] = sweep
    for k in ("ws_nt", "ws_nn", "ws_nt_mf4", "ws_nn_mf4", "ws_nt_gemm_only", "ws_nn_gemm_only", "r02_linear_nt", "r02_linear_nn",
              "hipblaslt_nt", "hipblaslt_nn"):
        if k in r:
            r[k + "_TBs"] = wb / r[k] / 1e6
    best_nt = min((v, k) for k, v in sweep.items() if k.startswith("nt") and isinstance(v, float))
    best_nn = min((v, k) for k, v in sweep.items() if k.startswith("nn") and isinstance(v, float))
    r["best_nt"], r["best_nn"] = best_nt, best_nn
    print(f"{name:8s} M={M} N={N} K={K} ws_nt {r['ws_nt']:.1f}us ({r['ws_nt_TBs']:.2f} TB/s; gemm "
          f"{r['ws_nt_gemm_only']:.1f}) ws_nn {r['ws_nn']:.1f}us ({r['ws_nn_TBs']:.2f}; gemm {r['ws_nn_gemm_only']:.1f}) "
          f"r02 {r.get('r02_linear_nt', 0):.1f}/{r.get('r02_linear_nn', 0):.1f} hipblaslt {r['hipblaslt_nt']:.1f}/"
          f"{r['hipblaslt_nn']:.1f} mf4 {r['ws_nt_mf4']:.1f}/{r['ws_nn_mf4']:.1f} best_nt {best_nt} best_nn {best_nn}", flush=True)
    out.append(r)
    del pool
    torch.cuda.empty_cache()
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/ws_bench.json", "w"), indent=1)
