"""CLI: the reference's dataset preparation (``dataset_preparation.ipynb``), offline.

    python -m hyperion.cli.prepare_data --base_dir . \
        [--wikitext_raw DIR_with_wiki.{train,valid,test}.raw] [--cifar_bin DIR_with_data_batch_*.bin]

Writes ``<base_dir>/data/processed/wikitext2_tokenized`` (HF save_to_disk layout, input_ids int32 /
attention_mask int8, 128 tokens, pad = eos) and ``<base_dir>/data/processed/cifar10_{train,test}.pt``
— the paths every reference trainer reads (``distributed_utils.py:135,149,224``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--base_dir", default=os.getcwd())
    ap.add_argument("--wikitext_raw", default=None)
    ap.add_argument("--cifar_bin", default=None)
    ap.add_argument("--max_length", type=int, default=128)
    a = ap.parse_args(argv)
    from hyperion.data.prepare import gpt2_tokenizer, prepare_cifar10, prepare_wikitext2, read_wikitext_raw

    out = os.path.join(a.base_dir, "data", "processed")
    report = {}
    if a.wikitext_raw:
        raw = {}
        for split, fname in (("train", "wiki.train.raw"), ("validation", "wiki.valid.raw"), ("test", "wiki.test.raw")):
            p = os.path.join(a.wikitext_raw, fname)
            if os.path.exists(p):
                raw[split] = read_wikitext_raw(p)
        tok = gpt2_tokenizer()
        report["wikitext2"] = prepare_wikitext2(raw, os.path.join(out, "wikitext2_tokenized"), tok, a.max_length)
        report["tokenizer"] = type(tok).__name__
    if a.cifar_bin:
        report["cifar10"] = prepare_cifar10(a.cifar_bin, out)
    print(json.dumps(report))
    return 0


if __name__ == "__main__":
    sys.exit(main())
