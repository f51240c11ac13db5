"""hipBLASLt on each ResNet-50 conv's implicit-GEMM shape (im2col excluded): the vendor GEMM's time
for [M = N*P*Q, K = C*R*S] x [K, N = K_out] in bf16 — a reference point for what a GEMM of the same
dimensions achieves on MI355X, next to the Hyperion conv kernels (bench/conv_shapes.py)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.bench.conv_shapes import resnet50_convs  # noqa: E402


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
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


rows = []
for sh in resnet50_convs(32):
    N, C, H, K, R, s, p = sh["N"], sh["C"], sh["H"], sh["K"], sh["R"], sh["stride"], sh["pad"]
    P = (H + 2 * p - R) // s + 1
    M, KK = N * P * P, C * R * R
    a = torch.randn(M, KK, device="cuda").bfloat16()
    b = torch.randn(KK, K, device="cuda").bfloat16()
    t = ev(lambda: torch.matmul(a, b))
    dy = torch.randn(M, K, device="cuda").bfloat16()
    t_w = ev(lambda: torch.matmul(dy.t(), a))  # weight-gradient GEMM [K, M] x [M, C*R*S]
    rows.append(dict(sh, M=M, Kred=KK, gemm_us=t, tflops=2 * M * KK * K / t / 1e6, wgrad_gemm_us=t_w))
    print(json.dumps(rows[-1]), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(rows, open("gpurun_out/conv_gemm_equiv.json", "w"), indent=1)
