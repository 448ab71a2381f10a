"""``nn.Linear`` for the bf16 transformer path with a leaner backward.

Under autocast a stock Linear costs, besides its three GEMMs, a bf16→fp32 cast
of the weight gradient and a generic ATen reduction (+ cast) for the bias
gradient — ~1/6 of the non-GEMM kernel time of BERT-base / GPT-2-small
(profiles/r1_*_prof22.txt). :class:`FusedLinear` (same parameters and
state_dict keys) computes

* dW in fp32 straight from our split-M MFMA wgrad GEMM (``gemm.hip``; the
  reduction over B·T rows is spread over the whole chip),
* db with the hand-written deterministic column-sum kernel (``colsum``, fp32),
* dX as the usual bf16 GEMM.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from .._ext import C as _C


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        w = weight.to(torch.bfloat16)
        b = bias.to(torch.bfloat16) if bias is not None else None
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        ctx.save_for_backward(x, w)
        ctx.wdtype = weight.dtype
        ctx.bdtype = bias.dtype if bias is not None else None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        if gy.dtype != torch.bfloat16:
            gy = gy.to(torch.bfloat16)
        g2 = gy.view(-1, gy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ w).view(x.shape)
        if ctx.needs_input_grad[1]:
            if g2.shape[1] % 64 == 0 and x2.shape[1] % 64 == 0:
                # our split-M MFMA wgrad GEMM (gemm.hip): the hipBLASLt tiles picked
                # for this K ≫ M,N shape leave most CUs idle (profiles/r1_bert_prof26.txt)
                dw = _C.conv1x1_wgrad(g2, x2.contiguous())
            else:
                dw = torch.mm(g2.t(), x2, out_dtype=torch.float32)
            if dw.dtype != ctx.wdtype:
                dw = dw.to(ctx.wdtype)
        if ctx.bdtype is not None and ctx.needs_input_grad[2]:
            db = _C.colsum(g2)
            if db.dtype != ctx.bdtype:
                db = db.to(ctx.bdtype)
        return dx, dw, db


class FusedLinear(nn.Linear):
    """``nn.Linear`` whose bf16 GPU forward/backward runs through :class:`_LinearFn`
    (fp32 weight/bias gradients without cast passes); plain ``nn.Linear``
    everywhere else (CPU, fp32 without autocast)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and self.in_features % 8 == 0 and self.out_features % 8 == 0 and (
                x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                              and torch.get_autocast_dtype("cuda") == torch.bfloat16)):
            return _LinearFn.apply(x, self.weight, self.bias)
        return super().forward(x)
