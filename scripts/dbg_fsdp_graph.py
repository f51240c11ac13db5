"""Debug: persistent FSDP step, eager vs SegmentedStep vs GraphedClosure (one rank) — losses and
first non-finite parameter per step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HYPERION_COMM"] = "torch"
import torch  # noqa: E402

from hyperion.models.simple_lm import SimpleTransformerLM  # noqa: E402
from hyperion.models.transformer import TransformerEncoderLayer  # noqa: E402
from hyperion.ops.optim import FusedAdam  # noqa: E402
from hyperion.parallel.fsdp import FSDP, MixedPrecision, transformer_auto_wrap_policy  # noqa: E402
from hyperion.train.segments import SegmentedStep  # noqa: E402
from hyperion.train.step import GraphedClosure  # noqa: E402


def run(mode, steps=4):
    torch.manual_seed(0)
    bf = torch.bfloat16
    lm = SimpleTransformerLM(vocab_size=512, emb_dim=128, n_heads=2, n_layers=2, ff_dim=256, dropout=0.0,
                             causal=True).cuda()
    m = FSDP(lm, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
             device_id=torch.device("cuda", 0), mixed_precision=MixedPrecision(bf, bf, bf), persistent=True)
    opt = FusedAdam(list(m.parameters()), lr=1e-3, weight_decay=0.01, adamw=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    data = [torch.randint(0, 512, (4, 33), device="cuda", generator=g) for _ in range(steps)]
    ids = data[0].clone()

    def body():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=bf):
            loss = m.forward_loss(ids[:, :-1], ids[:, 1:])
        loss.backward()
        tn = m.clip_grad_norm_(1.0)
        opt.step()
        return torch.stack([loss.detach().float(), tn.float()])

    st = {"seg": lambda: SegmentedStep(body, warmup=1, module=m), "closure": lambda: GraphedClosure(body, warmup=1,
                                                                                                    module=m),
          "eager": lambda: body}[mode]()
    out = []
    for i in range(steps):
        ids.copy_(data[i])
        if i == 0:
            body()
        r = st()
        torch.cuda.synchronize()
        bad = [n for n, p in enumerate(m.parameters()) if not torch.isfinite(p).all()]
        gbad = [n for n, p in enumerate(m.parameters()) if p.grad is not None and not torch.isfinite(p.grad).all()]
        out.append((r.tolist(), bad[:3], gbad[:3]))
    return out


for mode in ("eager", "closure", "seg"):
    try:
        print(mode, run(mode), flush=True)
    except Exception as e:  # keep going: the point is the comparison
        print(mode, "ERROR", repr(e)[:400], flush=True)
