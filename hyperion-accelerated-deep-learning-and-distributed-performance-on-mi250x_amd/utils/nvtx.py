"""roctx ranges (SURVEY §5.1 MI355X plan: ranges around fwd / bwd / comm / optimizer).

On ROCm ``torch.cuda.nvtx`` is backed by roctx, so rocprofv3 ``--marker-trace`` shows these
ranges.  Disabled unless ``HYPERION_ROCTX=1`` (a range push is a host call per event).
"""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = os.environ.get("HYPERION_ROCTX", "0") == "1"


def enabled() -> bool:
    return _ENABLED and torch.cuda.is_available()


def range_push(name: str) -> None:
    if enabled():
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:  # pragma: no cover - roctx missing
            pass


def range_pop() -> None:
    if enabled():
        try:
            torch.cuda.nvtx.range_pop()
        except Exception:  # pragma: no cover
            pass


@contextlib.contextmanager
def annotate(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()
