"""BatchNorm2d (+ReLU) (+residual add) for NHWC activations.

``BatchNormAct2d`` is an ``nn.BatchNorm2d`` subclass (identical parameters,
buffers and state_dict keys) whose forward optionally adds a residual and
applies ReLU. With ``fused=True`` on a GPU it runs the hand-written gfx950
kernels of ``csrc/kernels/batchnorm.hip`` through :class:`_BNActFn`; otherwise
it is the plain ATen composition (reference path, and the numerics oracle).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn
from torch.nn import functional as F

from .._ext import C as _C


class BatchNormAct2d(nn.BatchNorm2d):
    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, act: bool = True,
                 residual: bool = False, fused: bool = False):
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.act = act
        self.residual = residual
        self.fused = fused

    def _use_fused(self, x: torch.Tensor) -> bool:
        return (self.fused and x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)
                and x.is_contiguous(memory_format=torch.channels_last) and _C.bn_supported(x.shape[1]))

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, dual: bool = False,
                stats: Optional[torch.Tensor] = None):
        """``dual=True`` returns (y, y_alias): two autograd outputs over the same
        data for two consumers (next conv + next residual add); their gradients
        are summed inside this op's backward kernel instead of by a separate
        autograd add. ``stats``: (Σx, Σx²) fp32 [2*C] already accumulated by the
        producing GEMM's epilogue (:func:`.conv.conv1x1`); training mode only."""
        if self._use_fused(x):
            return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.num_batches_tracked,
                          self.training, self.momentum, self.eps, residual if self.residual else None, self.act,
                          dual, stats if self.training else None)
        y = super().forward(x)
        if self.residual and residual is not None:
            y = y + residual
        if self.act:
            y = F.relu(y, inplace=True)
        return (y, y) if dual else y


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, residual, act, dual,
                nbt=None, stats=None):
        # nbt (num_batches_tracked) is incremented inside the apply kernel
        y, mean, invstd, bits = _C.bn_act_fwd(x, weight, bias, running_mean, running_var, residual, training,
                                              float(momentum), float(eps), bool(act), nbt, stats)
        # with the 1-bit ReLU mask (residual + act, training) the backward never reads y
        ctx.save_for_backward(x, weight, bias, mean, invstd, y if bits.numel() == 0 else bits)
        ctx.bits = bits.numel() > 0
        ctx.has_res = residual is not None
        ctx.act = act
        ctx.training = training
        ctx.dual = dual
        if dual:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, gy, gy2=None):
        x, weight, bias, mean, invstd, y_or_bits = ctx.saved_tensors
        if gy is None:
            gy, gy2 = gy2, None
        y, bits = (x, y_or_bits) if ctx.bits else (y_or_bits, None)  # y unused when bits are given
        gx, gw, gb, gres = _C.bn_act_bwd(gy, gy2, x, weight, bias, mean, invstd, y, ctx.act, ctx.has_res,
                                         ctx.training, bits)
        return gx, gw, gb, None, None, None, None, None, (gres if ctx.has_res else None), None, None, None, None


def bn_act(x, weight, bias, running_mean, running_var, num_batches_tracked, training, momentum, eps, residual,
           act, dual: bool = False, stats=None):
    nbt = num_batches_tracked if (training and num_batches_tracked is not None) else None
    if nbt is not None and (nbt.device != x.device or nbt.dtype != torch.int64):
        nbt.add_(1)
        nbt = None
    return _BNActFn.apply(x, weight, bias, running_mean, running_var, training, momentum, eps, residual, act, dual,
                          nbt, stats)


class _BNResBNActFn(torch.autograd.Function):
    """relu(bn(x) + bn2(x2)) in training mode, both BatchNorms on statistics
    from their producing GEMMs' epilogues: the downsample branch's BN output is
    never materialised; backward reduces bn2's sums in bn's reduce pass."""

    @staticmethod
    def forward(ctx, x, weight, bias, x2, weight2, bias2, rm, rv, nbt, stats, rm2, rv2, nbt2, stats2, momentum, eps,
                momentum2, eps2, dual):
        y, mean, invstd, bits, mean2, invstd2 = _C.bn_resbn_act_fwd(
            x, weight, bias, rm, rv, nbt, stats, x2, weight2, bias2, rm2, rv2, nbt2, stats2, float(momentum),
            float(eps), float(momentum2), float(eps2))
        ctx.save_for_backward(x, weight, mean, invstd, bits, x2, weight2, mean2, invstd2)
        if dual:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, gy, gy2=None):
        x, weight, mean, invstd, bits, x2, weight2, mean2, invstd2 = ctx.saved_tensors
        if gy is None:
            gy, gy2 = gy2, None
        dx, dw, db, dx2, dw2, db2 = _C.bn_resbn_act_bwd(gy, gy2, x, weight, mean, invstd, bits, x2, weight2, mean2,
                                                        invstd2)
        return (dx, dw, db, dx2, dw2, db2) + (None,) * 13


def resbn_ok(bn: nn.BatchNorm2d, x: torch.Tensor, stats) -> bool:
    return (bn.training and bn.affine and bn.track_running_stats and bn.momentum is not None
            and stats is not None and stats.numel() == 2 * x.shape[1] and bn.weight.dtype == torch.float32
            and isinstance(bn, BatchNormAct2d) and bn._use_fused(x))


def bn_resbn_act(bn: "BatchNormAct2d", x: torch.Tensor, stats: torch.Tensor, bn2: "BatchNormAct2d",
                 x2: torch.Tensor, stats2: torch.Tensor, dual: bool = False):
    """``relu(bn(x) + bn2(x2))`` (training; ``stats``/``stats2`` = (Σ, Σ²) of x / x2
    from their GEMM epilogues) — same parameters, buffers and running-stat
    updates as ``bn(x, residual=bn2(x2))``."""

    def _nbt(m):
        t = m.num_batches_tracked
        if t is not None and (t.device != x.device or t.dtype != torch.int64):
            t.add_(1)
            return None
        return t

    return _BNResBNActFn.apply(x, bn.weight, bn.bias, x2, bn2.weight, bn2.bias, bn.running_mean, bn.running_var,
                               _nbt(bn), stats, bn2.running_mean, bn2.running_var, _nbt(bn2), stats2, bn.momentum,
                               bn.eps, bn2.momentum, bn2.eps, dual)


class BatchNormAct1d(nn.BatchNorm1d):
    """``nn.BatchNorm1d`` over [N, C] (+ReLU) on the same fused kernels: a
    row-major [N, C] tensor is NHWC with H = W = 1 (reference ConvNet's
    fc1 → BatchNorm1d(128) → ReLU, main.py:39-41)."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, act: bool = True,
                 fused: bool = False):
        super().__init__(num_features, eps=eps, momentum=momentum)
        self.act = act
        self.fused = fused

    def forward(self, x: torch.Tensor):
        if (self.fused and x.is_cuda and x.dim() == 2 and x.dtype in (torch.bfloat16, torch.float32)
                and x.is_contiguous() and _C.bn_supported(x.shape[1])
                and (self.training or self.track_running_stats)):
            return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.num_batches_tracked,
                          self.training, self.momentum, self.eps, None, self.act)
        y = super().forward(x)
        return F.relu(y) if self.act else y
