"""Native tiled GEMM vs vendor on the transformer FFN / projection shapes, with their epilogues
(bias, GELU + pre-activation aux, dropout): every (tile, split-K) candidate, hipGraph-timed.

    python scripts/gemm_probe.py [--out gpurun_out/gemm_probe.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.ops import _native  # noqa: E402
from conv_roofline import gtime  # noqa: E402

SHAPES = [  # name, M, N, K, act, dropout
    ("gpt2_fc1_gelu_drop", 2032, 3072, 768, 2, 0.1),
    ("gpt2_fc1_gelu", 2032, 3072, 768, 2, 0.0),
    ("gpt2_fc2", 2032, 768, 3072, 0, 0.0),
    ("gpt2_qkv", 2032, 2304, 768, 0, 0.0),
    ("gpt2_out", 2032, 768, 768, 0, 0.0),
    ("vit_fc1_gelu", 6304, 3072, 768, 2, 0.0),
    ("lm256_fc1_relu_drop", 4064, 2048, 256, 1, 0.1),
    ("llama_gateup_128tok", 128, 22016, 4096, 0, 0.0),  # Llama-2-7B LoRA forward (weight-streaming regime)
    ("llama_qkv_128tok", 128, 12288, 4096, 0, 0.0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/gemm_probe.json")
    a = ap.parse_args()
    C = _native.native()
    if os.environ.get("HYPERION_SPLITK_INKERNEL") is not None:  # A/B: 0 = the separate reduce kernel
        C.gemm_set_splitk_inkernel(int(os.environ["HYPERION_SPLITK_INKERNEL"]))
    rows = []
    for name, M, N, K, act, p in SHAPES:
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act == 2 else None
        rng = _native.rng_state(x.device) if p > 0 else None

        def ven():
            y = torch.addmm(b, x, w.t())
            if act == 1:
                y = torch.relu(y)
            elif act == 2:
                y = torch.nn.functional.gelu(y)
            if p > 0:
                y = C.dropout(y, p, rng)
            return y

        r = {"shape": name, "M": M, "N": N, "K": K, "act": act, "dropout": p,
             "vendor_us": round(gtime(ven), 2), "vendor_gemm_only_us": round(gtime(lambda: torch.addmm(b, x, w.t())), 2)}
        best = None
        for tile in (-1, 0, 1, 2, 4, 5, 6, 7):
            for sp in (-1, 1, 2, 3, 4):
                try:
                    us = gtime(lambda: C.gemm(x, w, bias=b, act=act, aux=aux, tile=tile, splits=sp, drop_p=p, rng=rng))
                except RuntimeError:
                    continue
                r[f"t{tile}_s{sp}"] = round(us, 2)
                if best is None or us < best[0]:
                    best = (round(us, 2), tile, sp)
        r["native_best"] = best
        r["plan"] = C.gemm_plan(M, N, K)
        rows.append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
