"""Micro-timings of the rank-r LoRA kernels at the Llama-2-7B shapes (M = 128 tokens, K = N = 4096,
r = 16, P = 3 / 1): per-call device time, with and without dropout, in a hipGraph of 50 calls."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

C = _native.native()
dev = "cuda"
bf = torch.bfloat16
M, K, r = 128, 4096, 16


def per_call_us(fn, n=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
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


res = {}
for P in (3, 1):
    x = torch.randn(M, K, device=dev, dtype=bf)
    A = [torch.randn(r, K, device=dev, dtype=bf) * 0.1 for _ in range(P)]
    B = [torch.randn(K, r, device=dev, dtype=bf) * 0.1 for _ in range(P)]
    dB = [torch.empty_like(b) for b in B]
    dA = [torch.empty_like(a) for a in A]
    t = torch.zeros(4, M, 4 * r, device=dev)  # split-partial stacks as the fused layer uses them
    du = torch.zeros(4, M, 4 * r, device=dev)
    z = torch.empty(M, 4 * r, device=dev)
    dy = torch.randn(M, P * K, device=dev, dtype=bf)
    rs = _native.rng_state(x.device)
    tv, uv = t[:, :, :P * r], du[:, :, :P * r]
    res[f"P{P}_down_nodrop"] = per_call_us(lambda: C.lora_down(x, A, tv))
    res[f"P{P}_down_drop"] = per_call_us(lambda: C.lora_down(x, A, tv, rs, 0.05))
    res[f"P{P}_bwd_t"] = per_call_us(lambda: C.lora_bwd_t(dy, K, B, dB, tv, uv, 2.0))
    res[f"P{P}_bwd_a_nodrop"] = per_call_us(lambda: C.lora_bwd_a(x, dA, uv))
    res[f"P{P}_bwd_a_drop"] = per_call_us(lambda: C.lora_bwd_a(x, dA, uv, rs, 0.05))
    res[f"P{P}_torch_fill"] = per_call_us(lambda: z.zero_())
    res[f"P{P}_torch_add"] = per_call_us(lambda: z.add_(1.0))
print(json.dumps(res), flush=True)
