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
if which.startswith("ct"):  # CustomTransformer eager step (baseline suite row), ct32 / ct16
    import time

    from hyperion.models.transformer import create_custom_transformer
    from hyperion.ops.optim import FusedAdam
    from hyperion.train.amp import cast_for_compute

    m = create_custom_transformer().cuda().train()
    if which == "ct16":
        cast_for_compute(m, torch.bfloat16)
    use_torch = os.environ.get("HYPERION_KERNELS") == "torch"
    opt = torch.optim.Adam(m.parameters(), lr=1e-3) if use_torch else FusedAdam(m.parameters(), lr=1e-3)
    xin = torch.rand(32, 16, 512, device="cuda")
    xin = xin.bfloat16() if which == "ct16" else xin
    tgt = torch.rand(32, 16, 512, device="cuda")

    def step():
        out = m(xin)
        loss = torch.nn.functional.mse_loss(out.float(), tgt)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        step()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tt = time.perf_counter() - t0
    print({"model": which, "kernels": os.environ.get("HYPERION_KERNELS", "hyperion"), "ms_per_step": tt / 50 * 1e3,
           "host_ms_per_step": th / 50 * 1e3}, flush=True)
else:
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
