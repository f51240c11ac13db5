"""Where the bf16 copy / colsum kernels of a transformer step come from: one eager ViT-B/16 (or
GPT-2) training step under torch.profiler with Python stacks; prints the top call sites of
aten::copy_ / to / contiguous.   python scripts/micro/copy_sources.py [vit|gpt2]"""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hyperion.bench import models as M  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "vit"
orig = M._timeit
cap = {}


def grab(step, steps, warmup):
    cap["step"] = step
    return orig(step, 1, 1)


M._timeit = grab
if which == "vit":
    M.bench_vit_step(checkpointing=False, steps=1, warmup=1)
else:
    M.bench_lm_step(precision="bf16", model="gpt2_small", batch=16, steps=1, warmup=1)
step = cap["step"]
step()
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
sites = Counter()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::_to_copy", "aten::clone", "aten::contiguous"):
        st = [f for f in (ev.stack or []) if "site-packages/torch" not in f][:4]
        sites[(ev.name, str(ev.input_shapes)[:80] + " | " + " <- ".join(st))] += 1
for (name, st), n in sites.most_common(25):
    print(n, name, st[:400])
