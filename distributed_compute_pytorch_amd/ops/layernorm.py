"""Fused LayerNorm (gfx950 HIP kernels, csrc/kernels/layernorm.hip).

``FusedLayerNorm`` is an ``nn.LayerNorm`` subclass (same parameters /
state_dict keys). On a GPU with a supported shape (last dim a multiple of 8,
≤ 4096, contiguous) it runs the hand-written kernels; under bf16 autocast the
activation stays bf16 (statistics and affine in fp32 registers) instead of
autocast's fp32 upcast of layer_norm. Elsewhere it is ``F.layer_norm``.
"""
from __future__ import annotations


import torch
from torch import nn
from torch.nn import functional as F

from .._ext import C as _C
from .linear import _acc_target, accumulating

# under no_sync add dγ / dβ into the existing .grad inside the backward kernel
# (False: leave it to autograd's AccumulateGrad; profiles/r1_ln_accum_ab74.txt)
_LN_ACCUM = True


class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_dtype):
        y, mean, rstd = _C.layer_norm_fwd(x, weight, bias, eps, out_dtype)
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.params = (weight, bias)
        ctx.accum = accumulating()
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        acc = None
        if _LN_ACCUM and weight is not None and bias is not None and ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            # under DistributedDataParallel.no_sync: add dγ / dβ into the fp32
            # .grad tensors in the finalize kernel (no AccumulateGrad adds; see
            # linear.accumulate_grads_in_place)
            D = torch.Size((x.shape[-1],))
            tw, tb = _acc_target(ctx, ctx.params[0], D), _acc_target(ctx, ctx.params[1], D)
            if tw is not None and tb is not None:
                acc = [tw, tb]
        dx, dw, db = _C.layer_norm_bwd(dy, x, weight, bias, mean, rstd, accumulate_into=acc)
        return dx, dw, db, None, None


def fused_layer_norm(x, normalized_shape, weight=None, bias=None, eps=1e-5):
    D = x.shape[-1]
    if x.is_cuda and len(normalized_shape) == 1 and _C.layer_norm_supported(D) and x.dtype in (torch.float32,
                                                                                             torch.bfloat16):
        out_dtype = None
        if torch.is_autocast_enabled() and x.dtype == torch.float32:
            # fp32 residual stream in, bf16 out: the cast is fused into the kernel
            out_dtype = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return _LNFn.apply(x.contiguous(), weight, bias, eps, out_dtype)
    return F.layer_norm(x, normalized_shape, weight, bias, eps)


class FusedLayerNorm(nn.LayerNorm):
    def forward(self, x):
        return fused_layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
