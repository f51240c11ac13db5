"""FSDP collectives_at_world_1 check: eager and segmented steps over NativeComm vs identity, per step."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from test_gpu_fsdp_graph import _lm  # noqa: E402


def run(coll, graphed, steps=4, autocast=True, clip=True):
    from hyperion.models.transformer import TransformerEncoderLayer
    from hyperion.ops.optim import FusedAdam
    from hyperion.parallel.fsdp import FSDP, MixedPrecision, transformer_auto_wrap_policy
    from hyperion.train.segments import SegmentedStep

    bf = torch.bfloat16
    m = FSDP(_lm(0), auto_wrap_policy=transformer_auto_wrap_policy({TransformerEncoderLayer}),
             device_id=torch.device("cuda", 0), mixed_precision=MixedPrecision(bf, bf, bf), persistent=True,
             collectives_at_world_1=coll)
    opt = FusedAdam(list(m.parameters()), lr=1e-3, weight_decay=0.01, adamw=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    data = [torch.randint(0, 512, (4, 33), device="cuda", generator=g) for _ in range(steps)]
    ids = data[0].clone()

    def body():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=bf, enabled=autocast):
            loss = m.forward_loss(ids[:, :-1], ids[:, 1:])
        loss.backward()
        if clip:
            m.clip_grad_norm_(1.0)
        opt.step()
        return loss.detach()

    st = SegmentedStep(body, warmup=1, module=m) if graphed else None
    from hyperion.train import segments as S
    orig = S.SegmentedGraph.capture
    info = {}

    def cap(self, b):
        torch.cuda.synchronize()
        before = [p.detach().clone() for p in m.parameters()]
        full_before = [g.full.detach().float().clone() for g in m.flat_groups()]
        r = orig(self, b)
        torch.cuda.synchronize()
        info["param_change_in_capture"] = max(float((p.detach() - q).abs().max()) for p, q in zip(m.parameters(), before))
        info["full_change_in_capture"] = max(float((g.full.detach().float() - q).abs().max())
                                             for g, q in zip(m.flat_groups(), full_before))
        info["segments"] = len(self.graphs)
        return r

    S.SegmentedGraph.capture = cap
    out = []
    for i in range(steps):
        ids.copy_(data[i])
        if i == 0:
            body()
            if not graphed:
                body()
        loss = st() if graphed else body()
        torch.cuda.synchronize()
        fin = all(bool(torch.isfinite(p).all()) for p in m.parameters())
        out.append((round(float(loss), 5), fin))
    if graphed:
        S.SegmentedGraph.capture = orig
        out.append(info)
    return out


s = socket.socket()
s.bind(("127.0.0.1", 0))
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), HYPERION_COMM="native")
s.close()
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for coll, graphed, ac, clip in [(False, False, False, True), (True, False, False, True), (False, True, False, True),
                                (True, True, False, True), (False, True, False, False), (True, True, False, False)]:
    print("coll", coll, "graphed", graphed, "autocast", ac, "clip", clip, run(coll, graphed, autocast=ac, clip=clip),
          flush=True)
dist.destroy_process_group()
