#!/bin/bash
# LM under FSDP on every GPU of this node (reference: 02_development/run_language_fsdp.sh).
# The reference turned the NCCL watchdog off and exported two timeout variables nothing reads;
# here the watchdog stays on (hyperion.utils.env.apply_defaults) and the process-group timeout is
# the launcher's --timeout.  Extra args are passed through (e.g. --max_steps 50 --precision bf16).
set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
export NCCL_COLLNET_ENABLE=0
NGPU=${NGPU:-$(python3 -c "import torch; print(max(1, torch.cuda.device_count()))")}
cd "$(dirname "$0")/.."
exec python3 -m torch.distributed.run --standalone --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
  -m hyperion.cli.run_distributed --model language_fsdp --epochs "${EPOCHS:-25}" "$@"
