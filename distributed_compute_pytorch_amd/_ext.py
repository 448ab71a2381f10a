"""Loader for the native extension ``_C``.

The extension is built in-tree (``python -m distributed_compute_pytorch_amd._build``).
If it is missing it is built on first import (set ``DCP_NO_AUTOBUILD=1`` to
forbid that). There is no pure-Python fallback: every GPU op of this package
runs the HIP code in ``_C`` or fails loudly.
"""
from __future__ import annotations

import fcntl
import importlib
import os

import torch  # noqa: F401  (load torch's HIP runtime / RCCL before _C)

from . import _build

_C = None


def _try_import():
    return importlib.import_module("distributed_compute_pytorch_amd._C")


def load():
    global _C
    if _C is not None:
        return _C
    try:
        _C = _try_import()
        return _C
    except ImportError as e:
        if os.environ.get("DCP_NO_AUTOBUILD") == "1":
            raise ImportError(
                "distributed_compute_pytorch_amd native extension _C is not built; run "
                "`python -m distributed_compute_pytorch_amd._build`"
            ) from e
    lock_path = _build.REPO / "build" / ".build.lock"
    lock_path.parent.mkdir(parents=True, exist_ok=True)
    with open(lock_path, "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            _C = _try_import()
        except ImportError:
            _build.build()
            importlib.invalidate_caches()
            _C = _try_import()
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)
    return _C


C = load()
