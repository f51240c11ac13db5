"""Seeding.  The reference never seeds anything (SURVEY §4 "Seeds") although README.md:143 claims
reproducible seeds; every Hyperion trainer/bench calls this."""
from __future__ import annotations

import os
import random

import numpy as np
import torch


def seed_everything(seed: int = 0, rank: int = 0) -> int:
    s = int(seed) + int(rank)
    random.seed(s)
    np.random.seed(s % (2**32))
    torch.manual_seed(s)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(s)
    os.environ.setdefault("PYTHONHASHSEED", str(s))
    return s
