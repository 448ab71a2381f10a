"""Fused ResNet stem: conv 7x7/2 (3 -> C) + BatchNorm (training) + ReLU +
max-pool 3x3/2/1 as one autograd node (csrc/kernels/stem.hip, the stem GEMM in
gemm.hip).

Forward: the fp32 (or bf16) image is cast + zero-padded to a 4-channel bf16
NHWC copy, the conv runs as an MFMA implicit GEMM whose epilogue accumulates
the BN sums, and ONE pass applies BN + ReLU + max-pool (uint8 arg-max, and the
BN input at the arg-max for the backward). Backward: the BN reduction runs over
the 4x smaller pooled map, ONE gather pass writes the conv-output gradient,
and the weight gradient is the split-M MFMA weight-gradient GEMM reading the
same padded image (receptive fields gathered straight from Xp, no im2col), so
no vendor kernel runs in the stem — which also keeps it HIP-graph safe (the
MIOpen backward-weights solvers for stride-2 convs are not: their output
zeroing is not captured, tools/graph_nan_debug.py).

Same parameters / buffers as ``conv1`` + ``bn1`` (state_dict unchanged);
the running statistics and ``num_batches_tracked`` update like
``nn.BatchNorm2d`` in training mode.
"""
from __future__ import annotations

import torch

from .._ext import C as _C


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, nbt, momentum, eps, dual):
        H, W = x.shape[2], x.shape[3]
        xp, _ = _C.stem_prep(x, False)
        wm = _C.stem_weight(weight)
        y, st = _C.stem_conv_fwd(xp, wm, H, W)
        out, idx, xsel, mean, invstd = _C.stem_bn_pool_fwd(y, st, gamma, beta, running_mean, running_var, nbt,
                                                           float(momentum), float(eps))
        ctx.save_for_backward(xp, weight, y, idx, xsel, mean, invstd, gamma)
        ctx.dual = dual
        ctx.hw = (H, W)
        if dual:
            return out, out.view_as(out)
        return out

    @staticmethod
    def backward(ctx, gp, gp2=None):
        xp, weight, y, idx, xsel, mean, invstd, gamma = ctx.saved_tensors
        if gp is None:
            gp, gp2 = gp2, None
        gp = gp.to(torch.bfloat16)
        if gp2 is not None:
            gp2 = gp2.to(torch.bfloat16)
        dy, dg, db = _C.stem_bn_pool_bwd(gp, gp2, idx, xsel, y, mean, invstd, gamma)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = _C.stem_conv_wgrad(dy, xp, *ctx.hw)
            if weight.is_contiguous(memory_format=torch.channels_last) and not weight.is_contiguous():
                dw = dw.contiguous(memory_format=torch.channels_last)
        return None, dw, dg, db, None, None, None, None, None, None


def stem_supported(x: torch.Tensor, conv, bn, training: bool) -> bool:
    """Training, bf16 compute (autocast bf16 or a bf16 input: the stem GEMM is
    bf16 x bf16 -> fp32), the standard 7x7/2/3 conv without bias."""
    bf16 = x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                         and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    return (training and bf16 and x.is_cuda and not x.requires_grad and conv.kernel_size == (7, 7) and conv.stride == (2, 2)
            and conv.padding == (3, 3) and conv.bias is None and conv.groups == 1 and conv.dilation == (1, 1)
            and conv.weight.dtype == torch.float32 and bn.affine and bn.track_running_stats
            and bn.momentum is not None and _C.stem_supported(x, conv.out_channels))


def fused_stem(x: torch.Tensor, conv, bn, dual: bool = False):
    """maxpool3x3s2p1(relu(bn(conv(x)))) — (y, alias) when ``dual``."""
    nbt = bn.num_batches_tracked
    if nbt is not None and (nbt.device != x.device or nbt.dtype != torch.int64):
        nbt.add_(1)
        nbt = None
    return _StemFn.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, nbt, bn.momentum,
                         bn.eps, dual)
