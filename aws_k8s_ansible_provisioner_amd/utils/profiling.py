"""ROCTX ranges around engine phases (SURVEY §5 tracing/profiling row).

With ``AKAP_ROCTX=1`` the model runner brackets every prefill / decode step (and graph
capture) with a named range via torch.cuda.nvtx, which the ROCm build of PyTorch routes
to roctx -- ``rocprofv3 --marker-trace --kernel-trace`` then shows which kernels belong
to which engine phase.  Disabled (the default) it is a shared no-op context manager.
"""
from __future__ import annotations

import contextlib
import os

_ENABLED = os.environ.get("AKAP_ROCTX", "0") == "1"
_NULL = contextlib.nullcontext()


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


@contextlib.contextmanager
def _range(name: str):
    import torch
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def phase(name: str):
    return _range(name) if _ENABLED else _NULL
