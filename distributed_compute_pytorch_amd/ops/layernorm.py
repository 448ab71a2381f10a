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

import os

# residual dropout + LayerNorm as one kernel each way in the GPT-2 / BERT
# blocks (dropout_add_layer_norm); DCP_DADD_LN=0: separate dropout_add + LN
FUSE_DADD_LN = os.environ.get("DCP_DADD_LN", "1") != "0"

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
        dx, dw, db, _ = _C.layer_norm_bwd(dy, x, weight, bias, mean, rstd, accumulate_into=acc,
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


class _DropAddLNFn(torch.autograd.Function):
    """LayerNorm(res + dropout(branch)) in one kernel each way (LnDropAdd in
    ``ln_kernels.h``): the forward writes the new residual stream x and the LN
    output together; the backward writes dx (x's full gradient, the residual's
    gradient) and the branch's gradient dx · keep / (1 - p) together. The mask
    is dropout_add's (same Philox stream, same seed draw), so the fused and
    unfused blocks compute the same values. ``mode`` 0: y; 1: (y, x) — pre-LN,
    x is the next residual; 2: (y, alias of y) — post-LN."""

    @staticmethod
    def forward(ctx, branch, res, weight, bias, eps, out_dtype, p, rng, mode):
        seed, off = rng
        y, mean, rstd, xnew = _C.layer_norm_fwd(res, weight, bias, eps, out_dtype, branch=branch, p=p, seed=seed,
                                                offset_dev=off)
        ctx.save_for_backward(xnew, weight, bias, mean, rstd)
        ctx.params = (weight, bias)
        ctx.accum = accumulating()
        ctx.mode, ctx.p, ctx.seed, ctx.off = mode, p, seed, off
        if mode == 1:
            return y, xnew
        if mode == 2:
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, dy, d2=None):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        acc = None
        if _LN_ACCUM and weight is not None and bias is not None and ctx.needs_input_grad[2] and ctx.needs_input_grad[3]:
            D = torch.Size((x.shape[-1],))
            tw, tb = _acc_target(ctx, ctx.params[0], D), _acc_target(ctx, ctx.params[1], D)
            if tw is not None and tb is not None:
                acc = [tw, tb]
        dx, dw, db, gb = _C.layer_norm_bwd(dy, x, weight, bias, mean, rstd, accumulate_into=acc,
                                           grad_residual=d2 if ctx.mode == 1 else None,
                                           dy2=d2 if ctx.mode == 2 else None, drop_p=ctx.p, drop_seed=ctx.seed,
                                           drop_offset_dev=ctx.off, branch_grad=True)
        return gb, dx, dw, db, None, None, None, None, None


def dropout_add_layer_norm(branch, res, ln, p: float, training: bool, mode: int = 0):
    """``ln(res + dropout(branch, p))`` — mode 0: y; 1: (y, x) with x = res +
    dropout(branch) (pre-LN transformer blocks: x is the next residual); 2:
    (y, alias of y) (post-LN blocks). One fused kernel each way on the GPU
    (:class:`_DropAddLNFn`); elsewhere dropout_add then the LayerNorm."""
    from .dropout import _take_offset, dropout_add

    D = res.shape[-1]
    if (training and p > 0.0 and isinstance(ln, FusedLayerNorm) and res.is_cuda and len(ln.normalized_shape) == 1
            and branch.dtype == torch.bfloat16 and res.dtype in (torch.float32, torch.bfloat16)
            and branch.shape == res.shape and _C.layer_norm_supported(D)):
        out_dtype = None
        if torch.is_autocast_enabled() and res.dtype == torch.float32:
            out_dtype = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return _DropAddLNFn.apply(branch.contiguous(), res.contiguous(), ln.weight, ln.bias, ln.eps, out_dtype,
                                      float(p), _take_offset(res.device, res.numel()), mode)
    x = dropout_add(branch, res, p, training)
    if mode == 0:
        return ln(x)
    if isinstance(ln, FusedLayerNorm):
        return ln.forward_dual(x) if mode == 1 else ln.forward_dual_out(x)
    y = ln(x)
    return (y, x) if mode == 1 else (y, y)
