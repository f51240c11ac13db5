"""Debug: DDP graph step variants (split / native comm / shortcut fusion) vs eager reference."""
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hyperion.models.resnet import resnet18  # noqa: E402
from hyperion.ops.optim import FusedAdam  # noqa: E402
from hyperion.parallel import DDP  # noqa: E402
from hyperion.parallel.comm import NativeComm  # noqa: E402
from hyperion.train.amp import cast_for_compute  # noqa: E402
from hyperion.train.step import TrainStep  # noqa: E402
import hyperion.ops.conv as hconv  # noqa: E402

s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))


def make():
    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    return m


x = torch.rand(16, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.rand(16, 10, device="cuda")
for split, native, fuse, graph in [(False, True, True, True), (True, True, False, True), (True, True, True, True),
                                   (True, False, True, True), (False, False, True, False)]:
    hconv.FUSE_SHORTCUT_GRAD = fuse
    ref = make()
    ropt = FusedAdam(ref.parameters(), lr=1e-3, zero_grad_in_step=True)
    rstep = TrainStep(ref, ropt, torch.nn.MSELoss(), amp_dtype=None, graph=False)
    comm = NativeComm(torch.device("cuda", 0)) if native else None
    ddp = DDP(make(), bucket_cap_mb=2.0, first_bucket_mb=0.5, broadcast_buffers=False, buckets_at_world_1=True,
              comm=comm)
    dopt = FusedAdam(ddp.parameters(), lr=1e-3, zero_grad_in_step=True)
    dstep = TrainStep(ddp, dopt, torch.nn.MSELoss(), amp_dtype=None, graph=graph, warmup_iters=2,
                      split_backward=split)
    if graph:
        for _ in range(2):
            rstep(x, y)
    out = []
    for i in range(6):
        rl = rstep(x, y)
        dl = dstep(x, y)
        torch.cuda.synchronize()
        out.append(f"{rl.item():.5f}/{dl.item():.5f}")
    print(f"split={split} native={native} fuse={fuse} graph={graph} phase1={dstep._phase1} phase2={dstep._phase2}:",
          " ".join(out), flush=True)
dist.destroy_process_group()
