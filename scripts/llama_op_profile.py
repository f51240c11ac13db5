"""torch.profiler op census of a 2-layer Llama-2-7B-shaped LoRA step on the GPU (which aten ops launch kernels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from hyperion.models.llama import LlamaConfig, LlamaForCausalLM  # noqa: E402
from hyperion.models.lora import apply_lora  # noqa: E402
from hyperion.ops.optim import FusedAdam, clip_grad_norm_  # noqa: E402

cfg = LlamaConfig.llama2_7b()
cfg.num_hidden_layers = 2
dev = torch.device("cuda")
with torch.device(dev):
    m = LlamaForCausalLM(cfg).to(torch.bfloat16)
apply_lora(m)
params = [p for p in m.parameters() if p.requires_grad]
opt = FusedAdam(params, lr=1e-5, weight_decay=0.01, adamw=True)
ids = torch.randint(0, cfg.vocab_size, (1, 128), device=dev)
mask = torch.ones(1, 128, dtype=torch.long, device=dev)


def body():
    opt.zero_grad(set_to_none=False)
    loss = m(ids, attention_mask=mask, labels=ids).loss
    loss.backward()
    clip_grad_norm_(params, 1.0)
    opt.step()


for _ in range(3):
    body()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    body()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=60, max_name_column_width=30,
                                                       max_shapes_column_width=70))
