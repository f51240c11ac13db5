"""Graphed DDP trainers at world 2 (two gloo ranks sharing one GPU: the multi-GPU schedule
rehearsed with real inter-process collectives).

The captured step is a segmented hipGraph (train/segments.py): each gradient bucket's all-reduce
is an eager hole at the point inside the backward where the bucket completed, the BN-buffer
broadcast of ``broadcast_buffers=True`` a hole before the forward.  Checks, for the reference's
three DDP trainers (LM-256 fp16 AMP, ResNet-18 CIFAR fp16 AMP with BN buffers, Llama LoRA-DDP):

* the step really is graphed at world 2 (it fell back to eager);
* a dataset that is not a multiple of the batch: the short last batch runs eagerly beside the
  captured step (its gradients must stay the captured tensors and be all-reduced),
  over two epochs, and the replicas stay bit-identical (all-gathered checksums);
* step level (one small BN conv net, fp16 autocast, ``broadcast_buffers=True``): the segmented
  captured DDP step replays to the same parameters as the eager DDP step from the same start, on
  both ranks (trainer-level loss curves differ by the capture's warm-up steps, so the equality
  check lives here).

Reference: DDP trainers ``02_development/distributed_utils.py:132-278, 463-476`` (bucketed
all-reduce overlapped with backward, :159, :229, :475).
"""
import os
import tempfile

import pytest
import torch

from dist_utils import run_world
from parity import assert_losses_match, assert_update_parity, snapshot

pytestmark = pytest.mark.gpu


def _run(rank, world, which, graph):
    os.environ["HYPERION_COMM"] = "torch"  # gloo collectives between the two processes
    torch.cuda.set_device(0)
    from hyperion.train.distributed import (RunOptions, train_cifar_model_ddp, train_language_model_ddp,
                                            train_llama_fsdp)

    base = tempfile.mkdtemp(prefix=f"hyp_ddpg_{which}_{rank}_")
    opts = RunOptions(synthetic=True, seed=3, save=False, graph=graph, check_replicas=True, log=lambda s: None)
    if which == "lm":
        opts.dataset_size = 2 * 2 * 16 + 2 * 5  # 2 full batches of 16 per rank + a tail of 5
        r = train_language_model_ddp(rank, world, epochs=2, base_dir=base, opts=opts, batch_size=16)
    elif which == "cifar":
        opts.dataset_size = 2 * 2 * 16 + 2 * 3
        r = train_cifar_model_ddp(rank, world, epochs=2, base_dir=base, opts=opts, batch_size=16)
    else:
        from hyperion.models.llama import LlamaConfig

        cfg = LlamaConfig(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                          num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=256)
        opts.dataset_size = 2 * 3 * 2 + 2 * 1
        r = train_llama_fsdp(rank, world, epochs=2, base_dir=base, opts=opts, config=cfg, lora=True,
                             lora_parallel="ddp", batch_size=2, progress_every=0)
    return {"graphed": r["graphed"], "reason": r["graph_reason"], "replicas": r["replicas"],
            "losses": [h["loss"] for h in r["history"]]}


@pytest.mark.parametrize("which", ["lm", "cifar", "llama"])
def test_ddp_trainer_graphed_at_world_2(which):
    g = run_world(_run, 2, (which, True), timeout=600)
    for rank in (0, 1):
        assert g[rank]["graphed"], g[rank]["reason"]
        assert g[rank]["replicas"] and g[rank]["replicas"] > 0  # checksums compared and equal
        assert all(torch.isfinite(torch.tensor(v)) for v in g[rank]["losses"])
    assert g[0]["losses"] == g[1]["losses"]  # the epoch loss is all-reduced: one value on both ranks


def _ddp_steps(rank, world, steps, graphed):
    os.environ["HYPERION_COMM"] = "torch"
    torch.cuda.set_device(0)
    from hyperion.models.resnet import resnet18
    from hyperion.ops.optim import FusedAdam
    from hyperion.parallel.ddp import DDP
    from hyperion.train.amp import LossScaler
    from hyperion.train.segments import SegmentedStep

    torch.manual_seed(0)
    m = DDP(resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last), broadcast_buffers=True,
            bucket_cap_mb=8.0, first_bucket_mb=1.0)
    opt = FusedAdam(m.parameters(), lr=1e-3, weight_decay=0.01, adamw=True)
    scaler = LossScaler(enabled=True, device=torch.device("cuda"))
    g = torch.Generator(device="cuda").manual_seed(11 + rank)
    data = [(torch.randn(8, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last),
             torch.randint(0, 10, (8,), device="cuda", generator=g)) for _ in range(steps)]
    img, lbl = data[0][0].clone(), data[0][1].clone()
    before = snapshot(m.module.named_parameters())

    def body():
        opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=torch.float16):
            loss = torch.nn.functional.cross_entropy(m(img).float(), lbl)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        return loss.detach()

    body()  # gradients exist from here on (zeroed in place in every step)
    nseg = 0
    losses = []
    if graphed:
        st = SegmentedStep(body, warmup=1, module=m)
        for i in range(steps):
            img.copy_(data[i][0])
            lbl.copy_(data[i][1])
            if i == 0:
                body()
            losses.append(float(st()))
        nseg = st.seg.num_segments
    else:
        for i in range(steps):
            img.copy_(data[i][0])
            lbl.copy_(data[i][1])
            if i == 0:
                body()
                body()  # SegmentedStep: one warm-up call + the capture pass are steps too
            losses.append(float(body()))
    torch.cuda.synchronize()
    return {"state": {k: v.detach().float().cpu() for k, v in m.module.state_dict().items()},
            "params": {k for k, _ in m.module.named_parameters()}, "segments": nseg, "losses": losses,
            "before": before, "after": snapshot(m.module.named_parameters())}


def test_ddp_segmented_capture_matches_eager_two_ranks():
    g = run_world(_ddp_steps, 2, (3, True), timeout=600)
    e = run_world(_ddp_steps, 2, (3, False), timeout=600)
    assert g[0]["segments"] > 2 and g[1]["segments"] > 2  # buffer broadcast + bucket all-reduces are holes
    for k, v in g[0]["state"].items():
        if k in g[0]["params"]:  # parameters: identical replicas (BN running stats are per-rank after
            assert torch.equal(v, g[1]["state"][k]), k  # the last forward, as with torch DDP)
        else:  # BN running statistics
            torch.testing.assert_close(v, e[0]["state"][k], rtol=2e-2, atol=5e-3)
    for r in (0, 1):
        # the per-step losses and the parameter UPDATE from the same start (tests/parity.py: a
        # skipped optimizer step or a stale gradient fails this; the parameters alone would pass)
        assert_losses_match(g[r]["losses"], e[r]["losses"], rtol=1e-2, what=f"rank {r}")
        assert_update_parity(e[r]["before"], g[r]["after"], e[r]["after"], rel=2e-2, what=f"rank {r}")
