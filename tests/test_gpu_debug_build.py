"""The bounds-checked debug build (``_C_debug.so``: -O1 -g, HYP_DASSERT device checks) and the
per-op kernel check (HYPERION_KERNEL_CHECK=nan) run the tiled GEMM (fast and SAFE kernels, every layout) clean:
no device check fires, results match the release build."""
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
