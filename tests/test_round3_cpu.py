"""CPU checks of round-3 helpers: the RoPE cos/sin table the fused attention backward reads, the
split-graph dropout guard, and the layer-norm affine-dtype handling of the Python op."""
import math

import torch

from hyperion.ops.layernorm import layer_norm
from hyperion.ops.rope import rope_reference, rope_table
from hyperion.train.step import _has_dropout


def test_rope_table_matches_reference_rotation():
    S, D, theta = 37, 128, 10000.0
    t = rope_table(S, D, theta, "cpu")
    assert t.shape == (S, D // 2, 2) and t.is_contiguous()
    assert rope_table(S, D, theta, "cpu") is t  # cached
    # rotating with the table == rope_reference
    q = torch.randn(1, S, 1, D)
    cos, sin = t[..., 0], t[..., 1]
    x1, x2 = q[0, :, 0, : D // 2], q[0, :, 0, D // 2 :]
    rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
    ref, _ = rope_reference(q, q, None, theta)
    torch.testing.assert_close(rot, ref[0, :, 0], atol=1e-4, rtol=1e-4)
    # inv_freq as the kernels compute it (exp2 of -(2i/D) log2 theta)
    i = 5
    assert math.isclose(float(t[1, i, 0]), math.cos(2 ** (-(2 * i / D) * math.log2(theta))), rel_tol=1e-5)


def test_split_graph_dropout_guard():
    assert not _has_dropout(torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.ReLU()))
    assert _has_dropout(torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Dropout(0.1)))
    assert not _has_dropout(torch.nn.Sequential(torch.nn.Dropout(0.0)))

    class Attn(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.dropout_p = 0.1

    assert _has_dropout(torch.nn.Sequential(Attn()))


def test_layer_norm_mixed_affine_dtypes_fall_back_consistently():
    torch.manual_seed(0)
    x = torch.randn(6, 64)
    w = torch.rand(64) + 0.5
    b = torch.randn(64)
    ref = torch.nn.functional.layer_norm(x, (64,), w, b, 1e-5)
    # fp32 input with bf16 affine parameters: upcast path, same result up to bf16 rounding of w / b
    y = layer_norm(x, w.bfloat16(), b.bfloat16(), 1e-5)
    torch.testing.assert_close(y, torch.nn.functional.layer_norm(x, (64,), w.bfloat16().float(),
                                                                  b.bfloat16().float(), 1e-5), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(layer_norm(x, w, b, 1e-5), ref, atol=1e-5, rtol=1e-5)
