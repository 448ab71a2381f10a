"""Tracing ranges: roctx (rocprofv3 --marker-trace) + torch.profiler.

``trace_range("name")`` opens a roctx range (native, csrc/trace) and a
``torch.profiler.record_function`` scope, so the same region shows up in a
rocprofv3 marker trace and in a torch profiler timeline. DDP wraps its
forward in ``DistributedDataParallel.forward`` (the name upstream uses,
SURVEY §5.1); the Reducer emits ``dcp.reducer.bucket_allreduce`` /
``dcp.reducer.finalize`` natively. Set ``DCP_ROCTX=0`` to disable roctx.
"""
from __future__ import annotations

import contextlib

import torch

from .._ext import C as _C


@contextlib.contextmanager
def trace_range(name: str):
    _C.trace_push(name)
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        _C.trace_pop()


def mark(name: str):
    _C.trace_mark(name)


def roctx_available() -> bool:
    return bool(_C.trace_enabled())
