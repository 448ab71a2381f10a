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
    """``dual=True``: also returns an alias of x as a second output — the
    pre-LN residual stream's other consumer — whose gradient the backward adds
    into dx inside the LN backward kernel (no separate fp32 add of the two
    gradients of x: 25 per GPT-2 micro-step)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_dtype, dual=0):
        """dual 1: (y, alias of x) — pre-LN residual stream; dual 2: (y, alias
        of y) — post-LN, the output's two consumers' gradients are summed as
        the backward loads dy."""
        y, mean, rstd = _C.layer_norm_fwd(x, weight, bias, eps, out_dtype)
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.params = (weight, bias)
        ctx.accum = accumulating()
        ctx.dual = dual
        if dual == 1:
            return y, x.view_as(x)
        if dual == 2:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, dy, d2=None):
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
        dx, dw, db = _C.layer_norm_bwd(dy, x, weight, bias, mean, rstd, accumulate_into=acc,
                                       grad_residual=d2 if ctx.dual == 1 else None,
                                       dy2=d2 if ctx.dual == 2 else None)
        return dx, dw, db, None, None, None


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


def fused_layer_norm_dual(x, normalized_shape, weight=None, bias=None, eps=1e-5, alias_output: bool = False):
    """(layer_norm(x), x) where the gradients of both outputs meet inside the
    LN backward kernel (pre-LN transformer blocks: ``h, x = ln_dual(x)``,
    ``x = x + f(h)``). ``alias_output``: (y, y) instead — post-LN blocks, whose
    normalised output feeds both the next sublayer and its residual add."""
    D = x.shape[-1]
    if x.is_cuda and len(normalized_shape) == 1 and _C.layer_norm_supported(D) and x.dtype in (torch.float32,
                                                                                             torch.bfloat16):
        out_dtype = None
        if torch.is_autocast_enabled() and x.dtype == torch.float32:
            out_dtype = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            y, alias = _LNFn.apply(x.contiguous(), weight, bias, eps, out_dtype, 2 if alias_output else 1)
        return y, alias
    y = F.layer_norm(x, normalized_shape, weight, bias, eps)
    return y, (y if alias_output else x)


class FusedLayerNorm(nn.LayerNorm):
    def forward(self, x):
        return fused_layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)

    def forward_dual(self, x):
        """(self(x), alias of x) — see :func:`fused_layer_norm_dual`."""
        return fused_layer_norm_dual(x, self.normalized_shape, self.weight, self.bias, self.eps)

    def forward_dual_out(self, x):
        """(self(x), alias of self(x)) — see :func:`fused_layer_norm_dual`."""
        return fused_layer_norm_dual(x, self.normalized_shape, self.weight, self.bias, self.eps, alias_output=True)
