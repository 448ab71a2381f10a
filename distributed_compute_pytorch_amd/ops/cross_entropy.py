"""Fused softmax cross-entropy over large vocabularies (csrc/kernels/xent.hip).

Reads bf16 logits directly (no fp32 upcast / log-softmax materialisation),
one pass forward (loss + log-sum-exp per row), one pass backward.
Semantics of ``F.cross_entropy(logits, target, ignore_index, reduction,
label_smoothing)`` for 2-D logits.
"""
from __future__ import annotations

import torch
from torch.nn import functional as F

from .._ext import C as _C


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, reduction, label_smoothing):
        loss, lse = _C.cross_entropy_fwd(logits, target, ignore_index, label_smoothing)
        ctx.save_for_backward(logits, target, lse)
        ctx.ignore_index, ctx.reduction, ctx.ls = ignore_index, reduction, label_smoothing
        if reduction == "none":
            return loss
        if reduction == "sum":
            return loss.sum()
        count = (target != ignore_index).sum().clamp_min(1)
        ctx.count = count
        return loss.sum() / count

    @staticmethod
    def backward(ctx, g):
        logits, target, lse = ctx.saved_tensors
        if ctx.reduction == "none":
            dl = g.float()
        elif ctx.reduction == "sum":
            dl = g.float().reshape(1)
        else:
            dl = (g.float() / ctx.count).reshape(1)
        d = _C.cross_entropy_bwd(logits, target, lse, dl, ctx.ignore_index, ctx.ls)
        return d, None, None, None, None


def fused_cross_entropy(logits, target, ignore_index: int = -100, reduction: str = "mean",
                        label_smoothing: float = 0.0):
    if logits.is_cuda and logits.dim() == 2 and logits.dtype in (torch.bfloat16, torch.float32):
        if logits.stride(1) != 1:
            logits = logits.contiguous()
        with torch.autocast("cuda", enabled=False):
            return _XentFn.apply(logits, target, ignore_index, reduction, float(label_smoothing))
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index, reduction=reduction,
                           label_smoothing=label_smoothing)
