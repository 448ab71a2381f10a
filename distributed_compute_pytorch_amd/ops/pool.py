"""NHWC max-pool with uint8 arg-max and gather backward (csrc/kernels/pool.hip)."""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from .._ext import C as _C


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = _C.maxpool2d_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geom = (k, s, p)
        ctx.shape, ctx.dtype, ctx.device = x.shape, x.dtype, x.device
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        k, s, p = ctx.geom
        like = torch.empty(ctx.shape, dtype=ctx.dtype, device=ctx.device).contiguous(
            memory_format=torch.channels_last)
        return _C.maxpool2d_bwd(gy, idx, like, k, s, p), None, None, None


def fused_max_pool2d(x, kernel_size: int = 3, stride: int = 2, padding: int = 0):
    if _C.maxpool_supported(x, kernel_size, padding):
        return _MaxPoolFn.apply(x, kernel_size, stride, padding)
    return F.max_pool2d(x, kernel_size, stride, padding)


class FusedMaxPool2d(nn.MaxPool2d):
    """nn.MaxPool2d (square kernel, no dilation / ceil_mode) on the NHWC kernel."""

    def forward(self, x):
        k = self.kernel_size if isinstance(self.kernel_size, int) else self.kernel_size[0]
        s = self.stride if isinstance(self.stride, int) else self.stride[0]
        p = self.padding if isinstance(self.padding, int) else self.padding[0]
        if self.dilation in (1, (1, 1)) and not self.ceil_mode and not self.return_indices:
            return fused_max_pool2d(x, k, s, p)
        return super().forward(x)
