"""CLI: activation-checkpointing memory probes (reference memory_optimization.ipynb), peak-correct."""
from __future__ import annotations

import argparse
import json
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--kinds", default="lm,resnet18")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from hyperion.bench.memory import checkpoint_memory_probe

    res = {k: checkpoint_memory_probe(k, precision=a.precision) for k in a.kinds.split(",")}
    print(json.dumps(res, indent=2))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
