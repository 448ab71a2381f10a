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
import sys

import torch  # noqa: F401  (load torch's HIP runtime / RCCL before _C)

from . import _build

_C = None


def _try_import():
    return importlib.import_module("distributed_compute_pytorch_amd._C")


def _stale() -> str | None:
    """Why the in-tree ``_C`` does not match ``csrc/`` (None if it does, or if
    there is no source tree to compare against)."""
    so = _build.ext_path()
    if not so.exists() or not _build.CSRC.is_dir():
        return None
    want, have = _build.source_digest(), _build.embedded_digest(so)
    if have != want:
        return f"{so.name} was built from other sources (embedded digest {have}, csrc/ digest {want})"
    return None


def load():
    global _C
    if _C is not None:
        return _C
    why = _stale()
    if why is None:
        try:
            _C = _try_import()
            return _C
        except ImportError as e:
            why = f"import failed: {e}"
    if os.environ.get("DCP_NO_AUTOBUILD") == "1":
        raise ImportError(
            f"distributed_compute_pytorch_amd native extension _C is missing or stale ({why}); run "
            "`python -m distributed_compute_pytorch_amd._build`"
        )
    print(f"[dcp] rebuilding the native extension: {why}", flush=True)
    lock_path = _build.REPO / "build" / ".build.lock"
    lock_path.parent.mkdir(parents=True, exist_ok=True)
    with open(lock_path, "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            if _stale() is not None:
                raise ImportError("stale")
            _C = _try_import()
        except ImportError:
            if "distributed_compute_pytorch_amd._C" in sys.modules:
                # a mapped library cannot be replaced in place: the loader would
                # hand the old mapping back to the import after the rebuild
                raise ImportError(
                    f"distributed_compute_pytorch_amd._C is stale ({why}) and already loaded in this process; "
                    "rebuild it (`python -m distributed_compute_pytorch_amd._build`) and restart")
            _build.build()
            importlib.invalidate_caches()
            _C = _try_import()
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)
    return _C


C = load()
