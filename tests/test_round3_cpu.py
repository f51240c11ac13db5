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


def test_stem_space_to_depth_rewrite_is_the_strided_conv():
    """The 7x7/s2/p3 stem == a stride-1 R=4 conv over the space-to-depth input read as 64-element
    runs of 4 adjacent 16-channel pixels (the rewrite csrc/kernels/stem.hip + the kernels' 16-element
    pixel stride implement), forward and weight gradient (index-map backward), in fp64."""
    import torch.nn.functional as F

    from hyperion.ops.conv import stem_runs_reference, stem_s2d_reference, stem_weight, stem_weight_grad

    for (N, C, H, W) in [(2, 3, 32, 32), (1, 3, 33, 31), (1, 4, 17, 18), (1, 1, 9, 9)]:
        x = torch.randn(N, C, H, W, dtype=torch.float64)
        w = torch.randn(8, C, 7, 7, dtype=torch.float64, requires_grad=True)
        ref = F.conv2d(x, w, stride=2, padding=3)
        xs = stem_s2d_reference(x)
        assert xs.shape[1] == 16 and xs.is_contiguous(memory_format=torch.channels_last)
        w4 = stem_weight(w)
        assert w4.shape == (8, 64, 4, 1) and w4.is_contiguous(memory_format=torch.channels_last)
        out = F.conv2d(stem_runs_reference(xs), w4)
        torch.testing.assert_close(out, ref)
        g = torch.randn_like(ref)
        (gw,) = torch.autograd.grad((out * g).sum(), w)
        (gr,) = torch.autograd.grad((ref * g).sum(), w)
        torch.testing.assert_close(gw, gr)
        # the explicit index-map backward the native path uses == autograd through the gather
        w4d = w4.detach().requires_grad_(True)
        out2 = F.conv2d(stem_runs_reference(xs), w4d)
        (gw4,) = torch.autograd.grad((out2 * g).sum(), w4d)
        torch.testing.assert_close(stem_weight_grad(gw4.contiguous(memory_format=torch.channels_last), C), gr)
