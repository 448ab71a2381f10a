"""Step timers (HIP events) and rank-0 JSON-lines metrics."""
from __future__ import annotations

import json
import sys
import time
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch


class StepTimer:
    """Per-phase device timing with events; resolved lazily (no sync in the step)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending: List[tuple] = []
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            yield
        finally:
            e.record()
            self._pending.append((name, s, e))

    def resolve(self):
        for name, s, e in self._pending:
            e.synchronize()
            self.totals[name] = self.totals.get(name, 0.0) + s.elapsed_time(e)
            self.counts[name] = self.counts.get(name, 0) + 1
        self._pending.clear()
        return {k: self.totals[k] / self.counts[k] for k in self.totals}


class JsonLogger:
    def __init__(self, rank: int = 0, path: Optional[str] = None, stream=None):
        self.rank = rank
        self.fh = open(path, "a") if (path and rank == 0) else None
        self.stream = stream

    def log(self, **kv):
        if self.rank != 0:
            return
        kv.setdefault("ts", time.time())
        line = json.dumps(kv, sort_keys=True)
        if self.fh:
            self.fh.write(line + "\n")
            self.fh.flush()
        if self.stream is not None:
            print(line, file=self.stream, flush=True)


def print0(*a, rank: int = 0, **kw):
    if rank == 0:
        print(*a, **kw, file=sys.stdout, flush=True)
