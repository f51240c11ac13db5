"""torch.profiler op census of one training step (which aten ops / kernels cost GPU time).

python scripts/op_census.py {vit,llama2,lm,resnet50} [sort_key]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from hyperion.ops.optim import FusedAdam  # noqa: E402
from hyperion.train.amp import cast_for_compute  # noqa: E402

which = sys.argv[1]
sort_key = sys.argv[2] if len(sys.argv) > 2 else "self_cuda_time_total"
dev = torch.device("cuda")
torch.manual_seed(0)
if which == "vit":
    from hyperion.models.vit import vit_b_16

    m = vit_b_16().to(dev)
    cast_for_compute(m, torch.bfloat16)
    x = torch.rand(32, 3, 224, 224, device=dev).to(torch.bfloat16)
    y = torch.rand(32, 1000, device=dev)
    opt = FusedAdam(m.parameters(), lr=1e-3)

    def body():
        opt.zero_grad(set_to_none=True)
        torch.nn.functional.mse_loss(m(x).float(), y).backward()
        opt.step()
elif which == "resnet50":
    from hyperion.models import resnet50

    m = resnet50().to(dev).to(memory_format=torch.channels_last)
    cast_for_compute(m, torch.bfloat16)
    x = torch.rand(32, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.rand(32, 1000, device=dev)
    opt = FusedAdam(m.parameters(), lr=1e-3)

    def body():
        opt.zero_grad(set_to_none=True)
        torch.nn.functional.mse_loss(m(x).float(), y).backward()
        opt.step()
elif which == "lm":
    from hyperion.data.synthetic import SyntheticWikiText2
    from hyperion.models.simple_lm import GPT2_PAD, simple_lm_256

    m = simple_lm_256().to(dev)
    opt = FusedAdam(m.parameters(), lr=2e-4, weight_decay=0.01, adamw=True)
    ids = SyntheticWikiText2(n=32, seq_len=128, seed=0).input_ids.to(dev)
    x, yy = ids[:, :-1].contiguous(), ids[:, 1:].contiguous()

    def body():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m.forward_loss(x, yy, ignore_index=GPT2_PAD)
        loss.backward()
        opt.step()
else:
    raise SystemExit("use vit / resnet50 / lm")
for _ in range(3):
    body()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    body()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by=sort_key, row_limit=45, max_name_column_width=90,
                                                       max_shapes_column_width=80))
