"""Embedding lookup whose backward is HIP-graph capturable.

ATen's dense embedding backward on ROCm sorts the indices and sizes its
segment pass from a device->host read of the unique-index count (a rocPRIM
partition): inside a captured step that count is frozen at capture time, so a
replay with other token ids indexes out of bounds. Here the weight gradient is
one fp32 ``index_add_`` scatter (atomics, no host read, no data-dependent
sizes): same values up to fp32 summation order, capture-safe, and one kernel
instead of sort + segment passes. Tables of at most 8 rows (BERT's token
types, where the scatter's atomics all collide on 2 x 768 words: 200-400 µs)
use per-workgroup register sums instead (``_C.embedding_small_bwd``, ~10 µs).

The scatter is nondeterministic (fp32 atomics), so under
``torch.use_deterministic_algorithms(True)`` the lookup falls back to
``F.embedding``'s own deterministic sort-based backward whenever no stream
capture is in progress (a capture keeps the scatter: the sorted backward
cannot be captured at all).

Parity: ``torch.nn.Embedding`` (no padding_idx / max_norm / sparse) — same
parameter and state_dict key.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, weight):
        from .linear import accumulating

        ctx.save_for_backward(idx)
        ctx.shape = weight.shape
        ctx.wdtype = weight.dtype
        ctx.accum = accumulating()
        ctx.param = weight
        return F.embedding(idx, weight)

    @staticmethod
    def backward(ctx, g):
        from .linear import inplace_grad

        (idx,) = ctx.saved_tensors
        V, D = ctx.shape
        tgt = inplace_grad(ctx.param, ctx.shape, ctx.accum)
        if V <= 8 and D % 4 == 0 and g.is_cuda:
            # tiny tables (BERT's 2 token types): every row's atomics land on the
            # same V x D words — per-workgroup register sums instead (embedding.hip)
            from .._ext import C as _C

            out = tgt if tgt is not None else torch.zeros(V, D, device=g.device, dtype=torch.float32)
            _C.embedding_small_bwd(idx.reshape(-1).long().contiguous(), g.reshape(-1, D).float().contiguous(), out)
            if tgt is not None:
                return None, None
            return None, out if ctx.wdtype == torch.float32 else out.to(ctx.wdtype)
        if tgt is not None:  # scatter straight into the accumulated .grad (no zero fill, no add pass)
            tgt.index_add_(0, idx.reshape(-1), g.reshape(-1, D).float())
            return None, None
        gw = torch.zeros(V, D, device=g.device, dtype=torch.float32)
        gw.index_add_(0, idx.reshape(-1), g.reshape(-1, D).float())
        return None, gw if ctx.wdtype == torch.float32 else gw.to(ctx.wdtype)


def _capturing(t: torch.Tensor) -> bool:
    return t.is_cuda and torch.cuda.is_current_stream_capturing()


def embedding(idx: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if weight.requires_grad and torch.is_grad_enabled():
        if torch.are_deterministic_algorithms_enabled() and not _capturing(weight):
            return F.embedding(idx, weight)
        return _EmbeddingFn.apply(idx, weight)
    return F.embedding(idx, weight)


class FusedEmbedding(nn.Embedding):
    """``nn.Embedding`` with the capture-safe scatter backward."""

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        if (self.padding_idx is None and self.max_norm is None and not self.sparse
                and not self.scale_grad_by_freq):
            return embedding(idx, self.weight)
        return super().forward(idx)
