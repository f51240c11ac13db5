"""Fused linear-CE pass timings (in-graph) on the LM-256 head: LSE pass and gradient pass per tile
width, vs the vendor logits GEMM.  Output: gpurun_out/ce_sweep.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_shapes import gtime  # noqa: E402  (module runs its sweep on import only when executed)

C_ = _native.native()
rows = []
for N, E, V in [(4064, 256, 50257), (2032, 768, 50257)]:
    x = torch.randn(N, E, device="cuda").bfloat16()
    w = (torch.randn(V, E, device="cuda") * 0.05).bfloat16()
    b = torch.randn(V, device="cuda") * 0.1
    t = torch.randint(0, V, (N,), device="cuda")
    scale = torch.full((1,), 1.0 / N, device="cuda")
    lse, _ = C_.linear_ce_lse(x, w, b, t, -100)
    r = {"N": N, "E": E, "V": V, "vendor_logits": gtime(lambda: torch.nn.functional.linear(x, w, b.bfloat16()))}
    for bn in (64, 128):
        r[f"lse_bn{bn}"] = gtime(lambda: C_.linear_ce_lse(x, w, b, t, -100, bn))
        r[f"grad_full_bn{bn}"] = gtime(lambda: C_.linear_ce_grad(x, w, b, t, -100, lse, scale, 0, V, bn))
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    rows.append(r)
json.dump(rows, open("gpurun_out/ce_sweep.json", "w"), indent=1)
