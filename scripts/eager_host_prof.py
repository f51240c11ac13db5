"""Host-side (Python) profile of an eager model step: where the CPU time of the launch-bound eager
steps goes.  python scripts/eager_host_prof.py {vit,lm}  -> top functions by own and cumulative time."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hyperion.bench import models as M  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "vit"
orig = M._timeit
captured = {}


def grab(step, steps, warmup):
    captured["step"] = step
    return orig(step, steps, warmup)


M._timeit = grab
r = M.bench_vit_step(checkpointing=False, steps=5, warmup=3) if which == "vit" else M.bench_lm_step(
    precision="bf16", steps=5, warmup=3)
print(r, flush=True)
step = captured["step"]
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    step()
torch.cuda.synchronize()
pr.disable()
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(25)
    print(s.getvalue()[-6000:], flush=True)
