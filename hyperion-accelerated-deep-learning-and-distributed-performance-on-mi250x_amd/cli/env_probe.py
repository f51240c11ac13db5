"""Environment / device probe (reference C1: ``01_hardware_exploration.ipynb:151-168``,
``core_framework.ipynb:22-36``): versions, GPUs (arch, CUs, HBM), memory, RCCL; ``--json`` for a
machine-readable run manifest."""
from __future__ import annotations

import argparse
import json
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    from hyperion.ops import _native
    from hyperion.utils.device import device_info, get_gpu_memory, print_device_info

    info = device_info()
    info["memory"] = get_gpu_memory()
    info["hyperion_native"] = _native.loaded_path()
    if a.json:
        print(json.dumps(info, indent=2, default=str))
    else:
        print_device_info()
        print(f"native extension: {info['hyperion_native']}")
        print(f"memory: {info['memory']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
