"""The bounds-checked debug build (``_C_debug.so``: -O1 -g, HYP_DASSERT device checks) and the
per-op kernel check (HYPERION_KERNEL_CHECK=nan) run clean: no device check fires and results match
fp32 references.  Covered: the tiled GEMM (fast and SAFE kernels, every layout), flash
attention fwd/bwd, LayerNorm fwd/bwd (+ fused residual dropout), the implicit-GEMM conv family
(forward + BN statistics, stride-1 / stride-2 data gradient with the BN-backward epilogue, weight
gradient), the weight-streaming GEMM and the fused Llama LoRA layer (wstream + lora_fused)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "hyperion-accelerated-deep-learning-and-distributed-performance-on-mi250x_amd")

SCRIPT = r"""
import torch
from hyperion.ops import _native
C = _native.native()
assert C.debug_build, "expected the debug build"
assert isinstance(C, _native.CheckedModule)
torch.manual_seed(0)
for (M, N, K, at, bt) in [(392, 776, 200, False, False), (1000, 264, 1032, True, True), (512, 512, 512, False, True)]:
    a = torch.randn(K, M, device="cuda").bfloat16() if at else torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16() if bt else torch.randn(N, K, device="cuda").bfloat16()
    for tile in (0, 1, 2, 3):
        c = C.gemm(a, b, a_tr=at, b_tr=bt, out_dtype=torch.float32, tile=tile, splits=2)
        ref = (a.float().t() if at else a.float()) @ (b.float() if bt else b.float().t())
        assert (c - ref).abs().max().item() < 1e-2 * K ** 0.5, (M, N, K, at, bt, tile)
torch.cuda.synchronize()
print("DEBUG-BUILD-OK")
"""

SCRIPT_KERNELS = r"""
import torch
import torch.nn.functional as F
from hyperion.ops import _native
C = _native.native()
assert C.debug_build, "expected the debug build"
torch.manual_seed(0)
rel = lambda a, b: float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))

# flash attention (attention.hip): causal forward + backward against fp32 SDPA
from hyperion.ops.attention import attention
q, k, v = (torch.randn(2, 200, 4, 64, device="cuda").bfloat16().requires_grad_() for _ in range(3))
o = attention(q, k, v, causal=True)
o.float().square().sum().backward()
qr, kr, vr = (t.detach().float().transpose(1, 2).requires_grad_() for t in (q, k, v))
orf = F.scaled_dot_product_attention(qr, kr, vr, is_causal=True)
orf.square().sum().backward()
assert rel(o.transpose(1, 2), orf) < 2e-2 and rel(q.grad.transpose(1, 2), qr.grad) < 5e-2
print("attention ok", flush=True)

# LayerNorm (layernorm.hip) with a residual and the fused residual-branch dropout
from hyperion.ops.layernorm import layer_norm
x = torch.randn(777, 768, device="cuda").bfloat16().requires_grad_()
r = torch.randn(777, 768, device="cuda").bfloat16()
w = torch.randn(768, device="cuda").requires_grad_()
b = torch.randn(768, device="cuda").requires_grad_()
y = layer_norm(x, w, b, 1e-5, residual=r)
y.float().sum().backward()
yr = F.layer_norm((x.detach().float() + r.float()), (768,), w.detach(), b.detach(), 1e-5)
assert rel(y, yr) < 1e-2
layer_norm(x, w, b, 1e-5, residual=r, dropout_p=0.1).float().sum().backward()
print("layernorm ok", flush=True)

# conv family (conv_igemm.hip / conv_wgrad.hip / stem.hip) through the fused conv-BN-ReLU op
from hyperion.ops.batchnorm import BatchNormAct2d
from hyperion.ops.conv import conv_bn_act
for (cin, cout, hw, ksz, st) in [(64, 64, 28, 3, 1), (64, 128, 28, 3, 2), (128, 64, 14, 1, 1), (3, 64, 32, 7, 2)]:
    conv = torch.nn.Conv2d(cin, cout, ksz, st, ksz // 2, bias=False).cuda().bfloat16().to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(cout, act=True).cuda()
    xi = torch.randn(4, cin, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xi.requires_grad_(cin != 3)
    out = conv_bn_act(conv, bn, xi)
    out.float().square().mean().backward()
    ref = F.relu(F.batch_norm(F.conv2d(xi.detach().float(), conv.weight.float(), None, st, ksz // 2), None, None,
                              bn.weight, bn.bias, True))
    assert rel(out, ref) < 3e-2, (cin, cout, ksz, st, rel(out, ref))
    assert torch.isfinite(conv.weight.grad).all()
print("conv ok", flush=True)

# weight-streaming GEMM (wstream.hip): skinny x Wᵀ and x W against fp32
xs = torch.randn(128, 4096, device="cuda").bfloat16()
ws = (torch.randn(1024, 4096, device="cuda") * 0.02).bfloat16()
assert rel(C.ws_linear(xs, ws), xs.float() @ ws.float().t()) < 1e-2
xn = torch.randn(128, 1024, device="cuda").bfloat16()
assert rel(C.ws_linear(xn, ws, nn=True), xn.float() @ ws.float()) < 1e-2
print("wstream ok", flush=True)

# fused Llama LoRA layer (llama_fused.py: wstream epilogues + lora_fused.hip)
from hyperion.models.llama import LlamaConfig, LlamaForCausalLM
from hyperion.models.lora import apply_lora
from hyperion.ops.llama_fused import fuse_llama_weights
cfg = LlamaConfig.tiny(hidden_size=256, num_attention_heads=2, num_key_value_heads=2, intermediate_size=512)
m = LlamaForCausalLM(cfg).cuda().to(torch.bfloat16)
apply_lora(m, r=16, alpha=32, dropout=0.0)
fuse_llama_weights(m)
ids = torch.randint(0, cfg.vocab_size, (2, 64), device="cuda")
_native.reset_counters()
loss = m(ids, labels=ids).loss
loss.backward()
assert torch.isfinite(loss) and _native.counters().get("llama_fused_layer", 0) >= 1, _native.counters()
print("lora ok", flush=True)
torch.cuda.synchronize()
print("DEBUG-KERNELS-OK")
"""


def _run_debug(script):
    env = dict(os.environ, HYPERION_DEBUG_BUILD="1", HYPERION_KERNEL_CHECK="nan", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=400)
    return r.returncode, r.stdout + r.stderr


def test_debug_build_kernel_families_run_clean():
    so = os.path.join(PKG, "_C_debug.so")
    if not os.path.exists(so):
        pytest.skip("_C_debug.so not built (python -m hyperion.csrc.build --debug)")
    rc, out = _run_debug(SCRIPT_KERNELS)
    assert rc == 0, out[-3000:]
    assert "DEBUG-KERNELS-OK" in out
    assert "device check failed" not in out, out[-3000:]


def test_debug_build_runs_clean():
    so = os.path.join(PKG, "_C_debug.so")
    if not os.path.exists(so):
        pytest.skip("_C_debug.so not built (python -m hyperion.csrc.build --debug)")
    env = dict(os.environ, HYPERION_DEBUG_BUILD="1", HYPERION_KERNEL_CHECK="nan", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "DEBUG-BUILD-OK" in out
    assert "device check failed" not in out, out[-3000:]
