"""CPU-side behaviour of the fp32 path's modules (ops/conv_f32.py, ops/linear_f32.py): drop-in
state dicts, CPU calls on the PyTorch ops, routing predicates off the GPU."""
import torch
import torch.nn as nn
import torch.nn.functional as F


def test_conv2d_is_a_drop_in_nn_conv2d_on_cpu():
    from hyperion.ops.conv_f32 import Conv2d, f32_conv_ok

    torch.manual_seed(0)
    ref = nn.Conv2d(8, 16, 3, stride=2, padding=1)
    ours = Conv2d(8, 16, 3, stride=2, padding=1)
    ours.load_state_dict(ref.state_dict())
    assert set(ours.state_dict()) == set(ref.state_dict())
    x = torch.randn(2, 8, 9, 9)
    assert not f32_conv_ok(x, ours)  # CPU: the torch op runs
    torch.testing.assert_close(ours(x), ref(x))


def test_linear_f32_routing_is_gpu_and_size_gated():
    from hyperion.ops import linear_f32

    w = torch.randn(3072, 768)
    assert not linear_f32.applies(torch.randn(4, 768), w)  # CPU tensor
    assert linear_f32.MIN_MACS >= 1 << 20


def test_resnet_models_keep_torchvision_keys_with_native_conv():
    from hyperion.models import resnet50
    from hyperion.ops.conv_f32 import Conv2d

    m = resnet50(num_classes=10)
    convs = [mod for mod in m.modules() if isinstance(mod, nn.Conv2d)]
    assert convs and all(isinstance(c, Conv2d) for c in convs)
    keys = set(m.state_dict())
    assert "conv1.weight" in keys and "layer1.0.downsample.0.weight" in keys


def test_conv2d_f32_reference_oracle_matches_functional():
    from hyperion.ops.conv_f32 import conv2d_f32_reference

    x, w, b = torch.randn(1, 3, 8, 8), torch.randn(4, 3, 3, 3), torch.randn(4)
    torch.testing.assert_close(conv2d_f32_reference(x, w, b, 1, 1).float(), F.conv2d(x, w, b, 1, 1), rtol=1e-5,
                               atol=1e-5)
