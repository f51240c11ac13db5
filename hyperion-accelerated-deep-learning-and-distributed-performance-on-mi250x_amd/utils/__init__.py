"""Runtime utilities: device probe, env knobs, seeding, timers, memory stats, manifests."""
from .device import (  # noqa: F401
    device_info,
    get_device,
    get_gpu_memory,
    is_gfx950,
    local_rank,
    on_gpu,
)
from .seed import seed_everything  # noqa: F401
from .timers import EventTimer, WallTimer, cuda_sync  # noqa: F401
