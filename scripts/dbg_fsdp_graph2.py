"""Debug: which part of the captured persistent-FSDP step goes non-finite (forward / backward / clip /
optimizer), FSDP vs the bare model."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HYPERION_COMM"] = "torch"
import torch  # noqa: E402

from hyperion.models.simple_lm import SimpleTransformerLM  # noqa: E402
from hyperion.models.transformer import TransformerEncoderLayer  # noqa: E402
from hyperion.ops.optim import FusedAdam  # noqa: E402
from hyperion.parallel.fsdp import FSDP, MixedPrecision, transformer_auto_wrap_policy  # noqa: E402
from hyperion.train.step import GraphedClosure  # noqa: E402

bf = torch.bfloat16


def build(fsdp):
    torch.manual_seed(0)
    lm = SimpleTransformerLM(vocab_size=512, emb_dim=128, n_heads=2, n_layers=2, ff_dim=256, dropout=0.0,
                             causal=True).cuda()
    if not fsdp:
        return lm.to(bf), lm
    m = FSDP(lm, auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
             device_id=torch.device("cuda", 0), mixed_precision=MixedPrecision(bf, bf, bf), persistent=True)
    return m, lm


def run(fsdp, stage):
    m, inner = build(fsdp)
    opt = FusedAdam(list(m.parameters()), lr=1e-3, weight_decay=0.01, adamw=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    ids = torch.randint(0, 512, (4, 33), device="cuda", generator=g)

    def body():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=bf):
            loss = m.forward_loss(ids[:, :-1], ids[:, 1:])
        if stage == "fwd":
            return loss.detach().float().reshape(1)
        loss.backward()
        outs = [loss.detach().float().reshape(1)]
        if stage in ("clip", "opt"):
            outs.append(m.clip_grad_norm_(1.0).float().reshape(1) if fsdp else
                        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0).float().reshape(1))
        if stage == "opt":
            opt.step()
        return torch.cat(outs)

    e = body()
    st = GraphedClosure(body, warmup=1, module=m)
    r = [st().tolist() for _ in range(2)]
    torch.cuda.synchronize()
    gb = [n for n, p in enumerate(m.parameters()) if p.grad is not None and not torch.isfinite(p.grad).all()]
    pb = [n for n, p in enumerate(m.parameters()) if not torch.isfinite(p).all()]
    fb = [n for n, p in inner.named_parameters() if not torch.isfinite(p).all()][:3]
    return {"eager_fwd": e.tolist(), "graph": r, "grad_bad": gb[:4], "param_bad": pb[:4], "inner_bad": fb}


for fsdp in (False, True):
    for stage in ("fwd", "bwd", "clip", "opt"):
        try:
            print("fsdp" if fsdp else "bare", stage, run(fsdp, stage), flush=True)
        except Exception as ex:
            print("fsdp" if fsdp else "bare", stage, "ERROR", repr(ex)[:300], flush=True)
