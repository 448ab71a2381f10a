"""NHWC max-pool with uint8 arg-max and gather backward (csrc/kernels/pool.hip),
optionally fused with ReLU and channel dropout (the reference ConvNet's
relu → max_pool2d → Dropout2d, main.py:33-36)."""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from .._ext import C as _C


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, relu, drop_p, rng, dual=False):
        seed, off = rng if rng is not None else (0, None)
        y, idx = _C.maxpool2d_fwd(x, k, s, p, relu, drop_p, seed, off)
        ctx.save_for_backward(idx, off if off is not None else idx.new_empty(0))
        ctx.geom = (k, s, p, drop_p, seed)
        ctx.shape = tuple(x.shape)
        if dual:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, gy, gy2=None):
        idx, off = ctx.saved_tensors
        k, s, p, drop_p, seed = ctx.geom
        if gy is None:
            gy, gy2 = gy2, None
        gx = _C.maxpool2d_bwd(gy, idx, list(ctx.shape), k, s, p, drop_p, seed, off if off.numel() else None, gy2)
        return gx, None, None, None, None, None, None, None


def fused_max_pool2d(x, kernel_size: int = 3, stride: int = 2, padding: int = 0, dual: bool = False):
    """``dual=True`` returns (y, alias) — two autograd outputs whose gradients
    are summed inside the backward gather (a pooled map read by two convs)."""
    if _C.maxpool_supported(x, kernel_size, padding):
        return _MaxPoolFn.apply(x, kernel_size, stride, padding, False, 0.0, None, dual)
    y = F.max_pool2d(x, kernel_size, stride, padding)
    return (y, y) if dual else y


def relu_max_pool2d_dropout(x, kernel_size: int = 2, stride: int = None, padding: int = 0, p: float = 0.0,
                            training: bool = True):
    """Dropout2d_p(max_pool2d(relu(x))) in one kernel each way (NHWC bf16/fp32, C % 8 == 0);
    falls back to the ATen composition otherwise."""
    stride = kernel_size if stride is None else stride
    drop = p if training else 0.0
    if _C.maxpool_supported(x, kernel_size, padding):
        from .dropout import _take_offset

        rng = _take_offset(x.device, x.shape[0] * x.shape[1]) if drop > 0 else None
        return _MaxPoolFn.apply(x, kernel_size, stride, padding, True, float(drop), rng)
    return F.dropout2d(F.max_pool2d(F.relu(x), kernel_size, stride, padding), drop, training)


class FusedMaxPool2d(nn.MaxPool2d):
    """nn.MaxPool2d (square kernel, no dilation / ceil_mode) on the NHWC kernel."""

    def forward(self, x, dual: bool = False):
        k = self.kernel_size if isinstance(self.kernel_size, int) else self.kernel_size[0]
        s = self.stride if isinstance(self.stride, int) else self.stride[0]
        p = self.padding if isinstance(self.padding, int) else self.padding[0]
        if self.dilation in (1, (1, 1)) and not self.ceil_mode and not self.return_indices:
            return fused_max_pool2d(x, k, s, p, dual)
        y = super().forward(x)
        return (y, y) if dual else y


class _GlobalAvgPoolNHWC(torch.autograd.Function):
    """mean over H, W of a channels_last [N, C, H, W] tensor -> [N, C]. The
    backward writes the broadcast gradient straight into channels_last memory
    (one streaming write) — ATen's adaptive-avg-pool backward returns an NCHW
    gradient that the next NHWC kernel then has to transpose-copy (a strided
    51 M-element copy per ResNet-50 step at batch 512, ~150 µs)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        return (g / (H * W))[:, :, None, None].expand(N, C, H, W).contiguous(memory_format=torch.channels_last)


def global_avg_pool_flat(x: torch.Tensor) -> torch.Tensor:
    """``torch.flatten(nn.AdaptiveAvgPool2d(1)(x), 1)`` for channels_last x."""
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and x.requires_grad:
        return _GlobalAvgPoolNHWC.apply(x)
    return x.mean((2, 3))
