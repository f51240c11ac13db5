"""Per-call device time of the flash-attention kernels (forward; backward incl. its pre/post kernels)
at the shapes the model benches run, next to torch SDPA on the same [B, S, H, D] data.
Timed as a hipGraph of 20 calls (launch overhead amortised the way the graphed steps see it).
python scripts/attn_bench.py  -> one JSON line per shape."""
import faulthandler
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from hyperion.ops import _native  # noqa: E402

faulthandler.enable()
C = _native.native()
dev = "cuda"
bf = torch.bfloat16


def per_call_us(fn, n=20):
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
    best = 1e9
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return round(best, 2)


def eager_us(fn, n=20):
    """autograd backward does not capture (its engine thread); time it eagerly"""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1e3 / n, 2)


SHAPES = {  # name: (B, S, H, D, causal)
    "llama7b_s128": (1, 128, 32, 128, True),
    "vit_b16_b32": (32, 197, 12, 64, False),
    "gpt2_b8_s1024": (8, 1024, 12, 64, True),
    "lm_b32_s128": (32, 128, 4, 64, True),
    "long_b2_s4096_d128": (2, 4096, 16, 128, True),
}
for name, (B, S, H, D, causal) in SHAPES.items():
    q, k, v, do = (torch.randn(B, S, H, D, device=dev, dtype=bf) for _ in range(4))
    scale = 1.0 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, causal, scale, 0.0, None, None, True)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    print(name, "fwd", file=sys.stderr, flush=True)
    fwd = per_call_us(lambda: C.attn_fwd(q, k, v, causal, scale, 0.0, None, None, True))
    bwd = per_call_us(lambda: C.attn_bwd(do, q, k, v, o, lse, causal, scale, 0.0, None, None, dq, dk, dv))
    print(name, "sdpa", file=sys.stderr, flush=True)
    qt, kt, vt = (x.transpose(1, 2).detach().requires_grad_() for x in (q, k, v))
    sd_f = per_call_us(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
    ot = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
    dot = do.transpose(1, 2)
    sd_b = eager_us(lambda: torch.autograd.grad(ot, (qt, kt, vt), dot, retain_graph=True))
    # numerics vs the fp32 math reference
    ref = F.scaled_dot_product_attention(*(x.float().transpose(1, 2) for x in (q, k, v)), is_causal=causal)
    err = (o.float() - ref.transpose(1, 2)).abs().max().item()
    flops = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
    print(json.dumps({"shape": name, "B": B, "S": S, "H": H, "D": D, "causal": causal, "fwd_us": fwd, "bwd_us": bwd,
                      "sdpa_fwd_us": sd_f, "sdpa_bwd_us": sd_b, "fwd_tflops": round(flops / fwd / 1e6, 1),
                      "bwd_tflops": round(2.5 * flops / bwd / 1e6, 1), "fwd_max_err": err}), flush=True)
