"""ResNet-50 bench A/B with diagnostic variants (upper bounds; never a headline number).

    python scripts/resnet_variants.py <variant> [bench.py args...]

variants:
  base         bench.py as is
  side         weight gradients on the side stream (HYPERION_WGRAD_STREAM=1)
  nowgrad      weight-gradient kernels skipped (dW = an uninitialised tensor): the step time the
               backward would have if every weight gradient were fully hidden behind the dgrad chain
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

variant = sys.argv[1]
argv = sys.argv[2:]
if variant == "side":
    os.environ["HYPERION_WGRAD_STREAM"] = "1"

import torch  # noqa: E402

import hyperion.ops.conv as conv  # noqa: E402

if variant == "nowgrad":
    def _skip(dy, x, w, stride, padding, w_param=None):
        return torch.empty_like(w)

    conv._wgrad = _skip

import bench  # noqa: E402

sys.exit(bench.main(argv))
