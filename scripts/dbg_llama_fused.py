"""Localize fused-vs-module differences of the Llama LoRA layer (prints rel errors per tensor)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import hyperion.models.llama as L  # noqa: E402
from hyperion.models.lora import apply_lora  # noqa: E402
from hyperion.ops.llama_fused import fuse_llama_weights  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


torch.manual_seed(0)
cfg = L.LlamaConfig.tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=2, intermediate_size=512,
                         num_hidden_layers=1)
m = L.LlamaForCausalLM(cfg).cuda().to(torch.bfloat16)
apply_lora(m, r=16, alpha=32, dropout=0.0)
with torch.no_grad():
    for n, p in m.named_parameters():
        if ".lora_B." in n:
            p.normal_(0, 0.02)
fuse_llama_weights(m)
layer = m.model.layers[0]
Bz, S, H = 2, 64, 256
for case in ("first", "delta"):
    torch.manual_seed(1)
    stream = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    delta = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16, requires_grad=True) if case == "delta" else None
    gd = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16)
    gs = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16)
    res = {}
    import copy
    ref_layer = copy.deepcopy(layer).float()
    os.environ["HYPERION_KERNELS"] = "torch"
    sf = stream.detach().float().requires_grad_(True)
    df = delta.detach().float().requires_grad_(True) if delta is not None else None
    d, s2 = ref_layer(df, sf)
    torch.autograd.backward([d, s2], [gd.float(), gs.float()])
    res["ref"] = dict(d=d.detach(), s2=s2.detach(), dstream=sf.grad, **({"ddelta": df.grad} if df is not None else {}),
                      **{n: p.grad for n, p in ref_layer.named_parameters() if p.grad is not None})
    del os.environ["HYPERION_KERNELS"]
    for fused in (True, False):
        L.FUSED = fused
        for p in layer.parameters():
            p.grad = None
        stream.grad = None
        if delta is not None:
            delta.grad = None
        d, s2 = layer(delta, stream)
        torch.autograd.backward([d, s2], [gd, gs])
        res[fused] = dict(d=d.detach().clone(), s2=s2.detach().clone(), dstream=stream.grad.clone(),
                          **({"ddelta": delta.grad.clone()} if delta is not None else {}),
                          **{n: p.grad.clone() for n, p in layer.named_parameters() if p.grad is not None})
    for k in res[False]:
        print(case, k, "fused-vs-module", round(rel(res[True][k], res[False][k]), 5), "fused-vs-fp32",
              round(rel(res[True][k], res["ref"][k]), 5), "module-vs-fp32", round(rel(res[False][k], res["ref"][k]), 5),
              flush=True)
