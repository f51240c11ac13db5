"""Steady per-step time of the reference-API trainers on one GPU (world 1), hipGraph-captured steps vs
eager, next to the matching bench_models graphed step.  Synthetic data; the
per-step time comes from each run's manifest (steady epochs: the reference skip-⌊n/3⌋ rule), so it
includes the data loader.  python scripts/trainer_steps.py [which ...]  -> one JSON line per run."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("HYPERION_BASE_DIR", "/tmp/hyp_trainers")

from hyperion.train import distributed as D  # noqa: E402

BASE = os.environ["HYPERION_BASE_DIR"]


def latest_manifest():
    ms = sorted(glob.glob(os.path.join(BASE, "data", "distributed", "*_run.json")), key=os.path.getmtime)
    return json.load(open(ms[-1])) if ms else {}


RUNS = {
    "language_ddp": lambda o: D.train_language_model_ddp(0, 1, epochs=3, base_dir=BASE, opts=o),
    "cifar": lambda o: D.train_cifar_model_ddp(0, 1, epochs=3, base_dir=BASE, opts=o),
    "language_fsdp": lambda o: D.train_language_model_fsdp(0, 1, epochs=3, base_dir=BASE, opts=o),
    "gpt2_fsdp": lambda o: D.train_gpt2_fsdp(0, 1, epochs=3, base_dir=BASE, opts=o),
    "llama_lora": lambda o: D.train_llama_fsdp(0, 1, epochs=3, base_dir=BASE, opts=o, lora=True),
}
SIZES = {"language_ddp": 3200, "cifar": 6400, "language_fsdp": 3200, "gpt2_fsdp": 1600, "llama_lora": 60}

which = sys.argv[1:] or list(RUNS)
for name in which:
    for graph in (True, False):
        opts = D.RunOptions(synthetic=True, dataset_size=SIZES[name], save=False, graph=graph, num_workers=2)
        try:
            RUNS[name](opts)
            m = latest_manifest()
            print(json.dumps({"trainer": name, "graph": graph, "ms_per_step": m.get("ms_per_step"),
                              "samples_per_s": m.get("samples_per_s"), "precision": m.get("precision"),
                              "per_rank_batch": m.get("per_rank_batch")}), flush=True)
        except Exception as e:  # keep the other rows
            print(json.dumps({"trainer": name, "graph": graph, "error": repr(e)[:300]}), flush=True)
