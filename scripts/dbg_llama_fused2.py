"""Step-by-step fp32 recomputation of the fused Llama layer's backward from its own saved tensors."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import hyperion.models.llama as L  # noqa: E402
import hyperion.ops.llama_fused as LF  # noqa: E402
from hyperion.models.lora import apply_lora  # noqa: E402
from hyperion.ops.attention import attention_reference  # noqa: E402
from hyperion.ops.rope import rope_reference  # noqa: E402


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
LF.fuse_llama_weights(m)
layer = m.model.layers[0]
Bz, S, H, I = 2, 64, 256, 512
M = Bz * S
torch.manual_seed(1)
stream = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
gd = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16)
gs = torch.randn(Bz, S, H, device="cuda", dtype=torch.bfloat16)
LF.DEBUG = {}
d, s2 = layer(None, stream)
torch.autograd.backward([d, s2], [gd, gs])
D = LF.DEBUG
at, mlp = layer.self_attn, layer.mlp
f = lambda t: t.float()  # noqa: E731
Wg, Wu, Wd = f(mlp.gate_proj.weight), f(mlp.up_proj.weight), f(mlp.down_proj.weight)
# MLP backward from the fused forward's own gu
gu = f(D["gu"])
g, u = gu[:, :I].clone().requires_grad_(True), gu[:, I:].clone().requires_grad_(True)
hh = F.silu(g) * u
dhh = f(D["dd"]) @ Wd
hh.backward(dhh)
print("dgu", rel(D["dgu"][:, :I], g.grad), rel(D["dgu"][:, I:], u.grad))
dh2 = f(D["dgu"][:, :I]) @ Wg + f(D["dgu"][:, I:]) @ Wu
print("dh2", rel(D["dh2"], dh2))
# ln2 backward: s2 = a + s -> h2 = rmsnorm(s2) * w2
s2f = f(D["s2"]).clone().requires_grad_(True)
w2 = f(layer.post_attention_layernorm.weight)
h2 = s2f * torch.rsqrt(s2f.pow(2).mean(-1, keepdim=True) + cfg.rms_norm_eps) * w2
h2.backward(f(D["dh2"]))
dsum2 = s2f.grad + f(D["ds2"])
print("dsum2", rel(D["dsum2"], dsum2))
# o projection dgrad with LoRA
A_o, B_o = f(at.o_proj.lora_A["default"].weight), f(at.o_proj.lora_B["default"].weight)
c = 2.0
du_o = c * f(D["dsum2"]) @ B_o
print("du_o", rel(D["du_o"], du_o))
do = f(D["dsum2"]) @ f(at.o_proj.weight) + du_o @ A_o
print("do", rel(D["do"], do))
# attention backward (fp32 reference on the fused forward's q, k, v)
q5 = f(D["qkv"]).view(Bz, S, 3, 2, 128)
q, k, v = (q5[:, :, i].clone().requires_grad_(True) for i in range(3))
o = attention_reference(q, k, v, causal=True)
print("o fwd", rel(D["o"], o))
o.backward(f(D["do"]).view(Bz, S, 2, 128))
# rope backward: grad wrt pre-rope = inverse rotation
dqr, dkr = rope_reference(q.grad, k.grad, None)  # forward rotation; inverse below via negative positions
pos = -torch.arange(S, device="cuda")[None].expand(Bz, S)
dqi, dki = rope_reference(q.grad, k.grad, pos)
dq5 = D["dqkv"].view(Bz, S, 3, 2, 128)
print("dq(pre-rope)", rel(dq5[:, :, 0], dqi), "dk", rel(dq5[:, :, 1], dki), "dv", rel(dq5[:, :, 2], v.grad))
# qkv dgrad with LoRA
W = torch.cat([f(at.q_proj.weight), f(at.k_proj.weight), f(at.v_proj.weight)], 0)
dy = f(D["dqkv"])
As = [f(x.lora_A["default"].weight) for x in (at.q_proj, at.k_proj, at.v_proj)]
Bs = [f(x.lora_B["default"].weight) for x in (at.q_proj, at.k_proj, at.v_proj)]
du = torch.cat([c * dy[:, p * H:(p + 1) * H] @ Bs[p] for p in range(3)], 1)
print("du_qkv", rel(D["du_qkv"], du))
dh = dy @ W + sum(du[:, 16 * p:16 * (p + 1)] @ As[p] for p in range(3))
print("dh", rel(D["dh"], dh))
sf = f(D["s"]).clone().requires_grad_(True)
w1 = f(layer.input_layernorm.weight)
hh1 = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + cfg.rms_norm_eps) * w1
hh1.backward(f(D["dh"]))
print("dsum1", rel(D["dsum1"], sf.grad + f(D["dsum2"])))
