"""Row log-softmax on a wave64-per-row HIP kernel (csrc/kernels/xent.hip).

Parity: the reference ConvNet's ``F.log_softmax(x, dim=1)`` head
(main.py:45). Under autocast a bf16 input produces fp32
log-probabilities (autocast's rule for log_softmax) without a separate cast.
"""
from __future__ import annotations

import torch
from torch.nn import functional as F

from .._ext import C as _C


class _LogSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_dtype):
        y = _C.log_softmax_fwd(x, out_dtype)
        ctx.save_for_backward(y)
        ctx.xdtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        return _C.log_softmax_bwd(gy, y, ctx.xdtype), None


def fused_log_softmax(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    """log_softmax over the last dimension (``dim`` must name it)."""
    if dim < 0:
        dim += x.dim()
    if not (x.is_cuda and dim == x.dim() - 1 and x.dtype in (torch.float32, torch.bfloat16)):
        return F.log_softmax(x, dim=dim)
    out = x.dtype
    if torch.is_autocast_enabled() and x.dtype == torch.bfloat16:
        out = torch.float32
    with torch.autocast(x.device.type, enabled=False):
        return _LogSoftmaxFn.apply(x.contiguous(), out)
