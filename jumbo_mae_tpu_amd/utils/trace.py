"""Phase ranges for rocprofv3 / roctracer timelines.

``torch.cuda.nvtx`` is backed by roctx on ROCm builds of PyTorch, so these ranges show up in
``rocprofv3 --marker-trace`` (and in torch.profiler) around the data / forward / backward /
all-reduce / optimizer phases of a step.  Off by default (a range push is a host call per
phase); enable with ``JMAE_TRACE=1`` or ``set_enabled(True)`` (driver flag ``--trace-ranges``).
"""

from __future__ import annotations

import contextlib
import os

import torch

_enabled = os.environ.get("JMAE_TRACE", "0") == "1"


def set_enabled(v: bool) -> None:
    global _enabled
    _enabled = bool(v)


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def trace_range(name: str):
    if not _enabled or not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
