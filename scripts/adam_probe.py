"""FusedAdam (bf16 compute copies + fp32 masters) device time over the parameter shapes of GPT-2-small
and ViT-B/16, plain vs streaming (non-temporal) fp32-state loads/stores: one JSON line per case."""
import json
import sys

import torch

sys.path.insert(0, ".")
from hyperion.ops import FusedAdam, _native  # noqa: E402


def shapes(name):
    if name == "gpt2":
        s = [(50257, 768), (1024, 768)]
        for _ in range(12):
            s += [(2304, 768), (2304,), (768, 768), (768,), (3072, 768), (3072,), (768, 3072), (768,)]
        return s
    s = [(768, 3, 16, 16), (768,), (1, 197, 768), (1000, 768), (1000,)]
    for _ in range(12):
        s += [(2304, 768), (2304,), (768, 768), (768,), (3072, 768), (3072,), (768, 3072), (768,)]
    return s


C = _native.native()
for name in ("gpt2", "vit"):
    ps = [torch.nn.Parameter(torch.randn(*sh, device="cuda").bfloat16()) for sh in shapes(name)]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = FusedAdam(ps, lr=1e-4)
    n = sum(p.numel() for p in ps)
    for nt in (0, 1, 0, 1):
        C.adam_set_streaming(nt)
        opt.step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            opt.step()
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) / 10 * 1e3
        print(json.dumps({"model": name, "params_M": round(n / 1e6, 2), "streaming": nt, "us": round(us, 1),
                          "TBps_30B": round(n * 30 / us / 1e6, 2)}), flush=True)
    C.adam_set_streaming(0)
