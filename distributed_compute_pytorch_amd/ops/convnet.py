"""Fused feature extractor of the reference ConvNet (csrc/kernels/convnet.hip):
``flatten(Dropout2d(max_pool2d(relu(conv2(relu(conv1(x)))), 2)))`` for
[B, 1, 28, 28] fp32 input, one kernel forward and one (+ a small reduce)
backward, both convolutions on the fp32 MFMA. Reference: main.py:23-24, 32-37.
"""
from __future__ import annotations

import torch
from torch.nn import functional as F

from .._ext import C as _C

_GRAD_SPLITS = (64 * 288, 64, 288, 32)


class _FeaturesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, p, rng):
        seed, off = rng if rng is not None else (0, None)
        out, mask = _C.convnet_features_fwd(x, w1.detach(), b1.detach(), w2.detach(), b2.detach(), p, seed, off)
        ctx.save_for_backward(x, w1, b1, w2, mask)
        ctx.scale = 1.0 / (1.0 - p) if p > 0 else 1.0
        ctx.mark_non_differentiable(mask)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w1, b1, w2, mask = ctx.saved_tensors
        flat = _C.convnet_features_bwd(g, mask, x, w1.detach(), b1.detach(), w2.detach(), ctx.scale)
        dw2, db2, dw1, db1 = flat.split(_GRAD_SPLITS)
        return None, dw1.view(32, 1, 3, 3), db1, dw2.view(64, 32, 3, 3), db2, None, None


class _FC32Fn(torch.autograd.Function):
    """y = x·Wᵀ + b in fp32 on the MFMA (csrc/kernels/fc32.hip): forward with
    a K-split + deterministic reduce, backward = data gradient + weight
    gradient with the bias gradient summed in the same launch. The reference
    ConvNet's fc1 / fc2 (main.py:27-28, 39, 43)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return _C.fc32_fwd(x, w.detach(), None if b is None else b.detach())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        dx, dw, db = _C.fc32_bwd(g.contiguous(), x, w.detach(), bool(ctx.needs_input_grad[0]))
        return (dx if ctx.needs_input_grad[0] else None), dw, (db if ctx.has_b else None)


def fc32(x: torch.Tensor, linear) -> torch.Tensor:
    """``linear(x)`` for an fp32 ``nn.Linear`` on the fp32 MFMA kernels (2-D
    contiguous fp32 device input), else the module itself."""
    w, b = linear.weight, linear.bias
    if (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and w.dtype == torch.float32 and w.is_contiguous()
            and (b is None or (b.dtype == torch.float32 and b.is_contiguous()))):
        return _FC32Fn.apply(x.contiguous(), w, b)
    return linear(x)


def _fits(x, conv1, conv2) -> bool:
    ps = (conv1.weight, conv1.bias, conv2.weight, conv2.bias)
    return (_C.convnet_supported(x) and not x.requires_grad and all(
        p is not None and p.dtype == torch.float32 and p.is_contiguous() for p in ps)
            and tuple(conv1.weight.shape) == (32, 1, 3, 3) and tuple(conv2.weight.shape) == (64, 32, 3, 3))


def convnet_features(x: torch.Tensor, conv1, conv2, p: float = 0.0, training: bool = True) -> torch.Tensor:
    """[B, 9216] fp32 features of the reference ConvNet up to (and including)
    ``dropout1`` + flatten. Falls back to the ATen composition for other
    shapes / dtypes or when ``x`` itself needs a gradient."""
    drop = p if training else 0.0
    if x.is_cuda and _fits(x, conv1, conv2):
        from .dropout import _take_offset

        rng = _take_offset(x.device, x.shape[0] * 64) if drop > 0 else None
        return _FeaturesFn.apply(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, float(drop), rng)
    y = F.relu(conv1(x))
    y = F.max_pool2d(F.relu(conv2(y)), 2)
    return torch.flatten(F.dropout2d(y, drop, training), 1)
