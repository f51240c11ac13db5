"""PMC / STREAM target: the hand-written MFMA GEMM at 8192^3 bf16 and the STREAM add at 500M fp32
(each a few launches), plus an event-timed sweep of the STREAM launch modes (grid-stride vs one
tile per workgroup, non-temporal vs default stores) against torch's add.

    python scripts/hw_one.py [gemm|gemm_tiled|gemm_tiled_wgrad|stream|sweep]
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "gemm"
C = _native.native()


def ev(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / 1e3)
    return statistics.median(ts)


if what == "gemm":
    n = 8192
    g = torch.Generator(device="cuda").manual_seed(0)
    a = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).bfloat16()
    b = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).bfloat16()
    t = ev(lambda: C.gemm_nt(a, b, None, 1.0, 64), reps=5, warm=2)
    print(json.dumps({"gemm_nt_8192_bf16_TF": 2 * n ** 3 / t / 1e12}))
elif what == "gemm_tiled":  # gemm_tiles.hip 256x256 fast kernel, 8192^3 NT
    n = 8192
    g = torch.Generator(device="cuda").manual_seed(0)
    a = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).bfloat16()
    b = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).bfloat16()
    t = ev(lambda: C.gemm(a, b, tile=0, splits=1), reps=5, warm=2)
    print(json.dumps({"gemm_tiled_8192_bf16_TF": 2 * n ** 3 / t / 1e12}))
elif what == "gemm_tiled_wgrad":  # ViT-B/16 fc1 weight gradient: [3072 x 768] = dyᵀ x over 6304 tokens
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = (torch.rand(6304, 3072, device="cuda", generator=g) * 2 - 1).bfloat16()
    x = (torch.rand(6304, 768, device="cuda", generator=g) * 2 - 1).bfloat16()
    t = ev(lambda: C.gemm(dy, x, a_tr=True, b_tr=True, tile=1, splits=3), reps=20, warm=3)
    print(json.dumps({"gemm_tiled_vit_fc1_wgrad_TF": 2 * 6304 * 3072 * 768 / t / 1e12}))
elif what == "stream":
    n = 500_000_000
    x, y, z = torch.rand(n, device="cuda"), torch.rand(n, device="cuda"), torch.empty(n, device="cuda")
    mode = int(os.environ.get("STREAM_BLOCKS", "0"))
    nt = os.environ.get("STREAM_NT", "1") == "1"
    t = ev(lambda: C.stream(2, x, y, z, 3.0, nt, mode), reps=5, warm=2)
    print(json.dumps({"stream_add_500M_GBps": 12 * n / t / 1e9, "blocks": mode, "nt": nt}))
else:
    rows = []
    for n in (100_000_000, 500_000_000):
        x, y, z = torch.rand(n, device="cuda"), torch.rand(n, device="cuda"), torch.empty(n, device="cuda")
        rows.append({"n": n, "kernel": "torch_add", "GBps": 12 * n / ev(lambda: torch.add(x, y, out=z)) / 1e9})
        for blocks in (0, 2048, -1, -2, -4, -8):
            for nt in (True, False):
                t = ev(lambda: C.stream(2, x, y, z, 3.0, nt, blocks))
                rows.append({"n": n, "kernel": f"hyp_add_blocks{blocks}_nt{int(nt)}", "GBps": 12 * n / t / 1e9})
        del x, y, z
    for r in rows:
        print(json.dumps(r))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/stream_sweep.json", "w") as f:
        json.dump(rows, f, indent=1)
