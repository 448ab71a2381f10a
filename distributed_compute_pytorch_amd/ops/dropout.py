"""Counter-based Philox dropout (csrc/kernels/dropout.hip).

The mask is a function of (seed, offset, element index): nothing is stored,
the backward regenerates it. Every call draws its seed from torch's CPU
generator (``torch.manual_seed`` makes runs reproducible; SURVEY App. A14:
the reference seeds every rank identically). Inside a HIP-graph capture the
drawn seed is frozen into the graph, so the call also snapshots and advances
a per-device Philox counter tensor (two tiny captured kernels): every replay
reads a new counter value and draws fresh masks. Eager calls skip the counter.
``dropout_add(x, residual, p)`` fuses the transformer residual add.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from .._ext import C as _C

_OK = (torch.float32, torch.bfloat16)


_COUNTER = {}
# device index -> counters consumed so far by the step being captured inside
# batched_offsets (None: no batching, one snapshot + advance per call)
_BATCH = [None]


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class batched_offsets:
    """Context wrapped around a whole captured training step
    (``utils.graphs.CapturedStep``): the dropout calls inside read the device
    counter itself — each call has its own host seed, frozen into the graph,
    so calls of one replay draw independent streams — and ONE captured add at
    the end of the step advances the counter past every counter the step
    consumed, so the next replay draws fresh masks. Without it every call
    snapshots and advances the counter itself: two tiny graph nodes per
    dropout (96 per GPT-2 step, ~0.9 ms of replay time: NOTES §31)."""

    def __enter__(self):
        self._outer = _BATCH[0]
        _BATCH[0] = {}
        return self

    def __exit__(self, *exc):
        used, _BATCH[0] = _BATCH[0], self._outer
        if exc[0] is None:
            for key, n in used.items():
                if n:
                    _COUNTER[key].add_(n)  # captured: runs at the end of every replay
        return False


def _take_offset(device, n):
    """(seed, device offset or None) for a call consuming ceil(n / 4) Philox counters."""
    seed = int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())
    if device.type != "cuda" or not _capturing():
        _ensure_counter(device)
        return seed, None
    key = device.index
    base = _COUNTER.get(key)
    if base is None:
        raise RuntimeError("dropout inside a HIP-graph capture needs an eager warmup call first")
    if _BATCH[0] is not None:
        _BATCH[0][key] = _BATCH[0].get(key, 0) + (n + 3) // 4
        return seed, base
    used = base.clone()
    base.add_((n + 3) // 4)
    return seed, used


def _ensure_counter(device):
    if device.type == "cuda" and device.index not in _COUNTER:
        _COUNTER[device.index] = torch.zeros(1, dtype=torch.int64, device=device)


class _DropFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, p, rng):
        seed, off = rng
        ctx.p, ctx.seed, ctx.has_res, ctx.xdtype, ctx.off = p, seed, residual is not None, x.dtype, off
        return _C.dropout_fwd(x, residual, p, seed, 0, None, off)

    @staticmethod
    def backward(ctx, gy):
        gx = _C.dropout_fwd(gy.contiguous(), None, ctx.p, ctx.seed, 0, ctx.xdtype, ctx.off)
        return gx, (gy if ctx.has_res else None), None, None


class _FeatDropFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, rng):
        seed, off = rng
        ctx.p, ctx.seed, ctx.off = p, seed, off
        return _C.feature_dropout_fwd(x, p, seed, 0, off)

    @staticmethod
    def backward(ctx, gy):
        return _C.feature_dropout_fwd(gy.contiguous(), ctx.p, ctx.seed, 0, ctx.off), None, None


def _usable(x):
    return x.is_cuda and x.dtype in _OK and x.is_contiguous()


def fused_dropout(x, p: float = 0.5, training: bool = True):
    if not training or p == 0.0:
        return x
    if _usable(x):
        return _DropFn.apply(x, None, float(p), _take_offset(x.device, x.numel()))
    return F.dropout(x, p, training)


def dropout_add(x, residual, p: float = 0.1, training: bool = True):
    """residual + dropout(x) in one pass."""
    if not training or p == 0.0:
        return residual + x
    if _usable(x) and residual.shape == x.shape and residual.dtype in _OK:
        return _DropFn.apply(x, residual.contiguous(), float(p), _take_offset(x.device, x.numel()))
    return residual + F.dropout(x, p, training)


def fused_feature_dropout(x, p: float = 0.5, training: bool = True):
    if not training or p == 0.0:
        return x
    if _usable(x) and x.dim() >= 3:
        return _FeatDropFn.apply(x, float(p), _take_offset(x.device, x.shape[0] * x.shape[1]))
    return F.dropout2d(x, p, training)


class FusedDropout(nn.Dropout):
    def forward(self, x):
        return fused_dropout(x, self.p, self.training)


class FusedDropout2d(nn.Dropout2d):
    def forward(self, x):
        return fused_feature_dropout(x, self.p, self.training)
