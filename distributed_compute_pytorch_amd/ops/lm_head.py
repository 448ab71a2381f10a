"""Tied LM head + softmax cross-entropy on our kernels.

``loss = F.cross_entropy(x @ Wᵀ + b, target)`` for a vocabulary-sized W (GPT-2's
tied ``wte`` [50257, 768], BERT's MLM head over the word embeddings [30522,
768]) as one autograd node:

* the bf16 weight and its transpose come from the model's
  :class:`~.linear.LinearWeightPrep`, padded with zero rows to ``Vp`` — the
  next multiple of 64 — so the vocabulary GEMMs take our kernels' shapes (no
  per-micro-step fp32→bf16 cast of the 38.6 M-parameter embedding);
* forward: logits [M, Vp] on the autotuned GEMM (256×256 ping-pong / 128×128
  ring / hipBLASLt), then the one-pass cross-entropy over the first V columns
  (``xent.hip``; the pad columns are never read) — or, without a bias, the
  ping-pong GEMM whose epilogue also emits each row's softmax partials
  (``gemm_pp.hip`` EPI 7), merged by a small kernel: the loss then costs no
  pass over the [M, Vp] logits (the autotune times GEMM + loss together);
* backward: the cross-entropy gradient is written IN PLACE over the logits,
  pad columns zeroed (no second [M, Vp] buffer), the data gradient is dL·W on
  the autotuned GEMM with K = Vp, and the fp32 weight gradient comes from our
  split-M wgrad GEMM straight into ``W.grad`` (only its first V rows; no bf16
  dW, no cast, no separate AccumulateGrad add — the tied embedding's two
  gradient contributions meet in one fp32 buffer).

Reference parity: the Linear + log_softmax / NLL head of ``main.py:27-28,43-44``
 at the BASELINE transformer configs' vocabulary size.
"""
from __future__ import annotations

import torch
from torch.nn import functional as F

from .._ext import C as _C
from .cross_entropy import fused_cross_entropy
from . import linear as _lin
from .linear import _pick, _pp_bias_ok, _pp_ok, accumulating, inplace_grad, prepped_linear


def padded_vocab(v: int) -> int:
    """Rows of the padded head weight: the next multiple of 64."""
    return (v + 63) // 64 * 64


_ZERO_BIAS: dict = {}


def _zero_bias(n: int, device) -> torch.Tensor:
    key = (n, device)
    z = _ZERO_BIAS.get(key)
    if z is None:
        z = _ZERO_BIAS[key] = torch.zeros(n, device=device, dtype=torch.float32)
    return z


class _LMHeadXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, target, wb, wt, ignore_index):
        V, K = weight.shape
        Vp = wb.shape[0]
        x2 = x.reshape(-1, K)
        if x2.dtype != torch.bfloat16:
            x2 = x2.to(torch.bfloat16)
        x2 = x2.contiguous()
        M = x2.shape[0]
        b32 = None
        if bias is not None:
            b32 = F.pad(bias.detach().float(), (0, Vp - V))
        tg = target.reshape(-1)
        if tg.dtype != torch.int64:
            tg = tg.long()

        def then_xent(gemm):  # a logits GEMM followed by the one-pass cross-entropy kernel
            def run():
                lg = gemm()
                return (lg,) + tuple(_C.cross_entropy_fwd(lg, tg, ignore_index, 0.0, V))
            return run

        # each candidate yields (logits, per-row loss, lse), so the autotune
        # weighs the GEMM together with the loss's cost: "pp_xent" takes the
        # softmax partials from the GEMM epilogue (no pass over the logits)
        cands = {}
        if b32 is None and Vp % 8 == 0 and _pp_ok(M, Vp, K):
            cands["pp_xent"] = lambda: tuple(_C.lm_head_xent_fwd(x2, wb, tg, ignore_index, V))
        if _pp_ok(M, Vp, K) and (b32 is None or _pp_bias_ok(Vp)):
            cands["pp"] = then_xent(lambda: _C.gemm_pp(x2, wb, b32, 0)[0])
        if K <= 4096 and K % 64 == 0:
            cands["ring"] = then_xent(
                lambda: _C.linear_fwd(x2, wb, b32 if b32 is not None else _zero_bias(Vp, x2.device), 0)[0])
        cands["hipblaslt"] = then_xent(
            lambda: F.linear(x2, wb, b32.to(torch.bfloat16) if b32 is not None else None))
        c = _pick(("head_xent", M, K, Vp), cands)
        logits, loss, lse = cands[c]()
        count = (tg != ignore_index).sum().clamp_min(1)
        ctx.save_for_backward(x2, logits, lse, tg, wb, wt, count)
        ctx.ignore_index, ctx.V, ctx.accum = ignore_index, V, accumulating()
        ctx.params = (weight, bias)
        ctx.xshape, ctx.xdtype = x.shape, x.dtype
        return loss.sum() / count

    @staticmethod
    def backward(ctx, g):
        if getattr(ctx, "consumed", False):
            raise RuntimeError("lm_head_cross_entropy: a second backward through the same graph is not supported "
                               "(the first one overwrote the saved logits with their gradient)")
        ctx.consumed = True
        x2, logits, lse, tg, wb, wt, count = ctx.saved_tensors
        weight, bias = ctx.params
        V = ctx.V
        M, K = x2.shape
        Vp = wb.shape[0]
        dl = (g.float() / count).reshape(1)
        d = _C.cross_entropy_bwd(logits, tg, lse, dl, ctx.ignore_index, 0.0, V, True)  # [M, Vp], pad cols 0
        dx = dw = db = None
        n = ctx.needs_input_grad
        if n[0]:
            cands = {}
            if _pp_ok(M, K, Vp):
                cands["pp"] = lambda: _C.gemm_pp(d, wt)[0]
            cands["hipblaslt"] = lambda: d @ wb
            c = _pick(("head_dgrad", M, Vp, K), cands)
            dx = cands[c]().view(ctx.xshape)
            if dx.dtype != ctx.xdtype:
                dx = dx.to(ctx.xdtype)
        if n[1]:
            tgt = inplace_grad(weight, weight.shape, ctx.accum)
            dw = _head_wgrad(d, x2, V, tgt)
            if tgt is not None:
                dw = None  # added into weight.grad by the GEMM itself
            elif dw.dtype != weight.dtype:
                dw = dw.to(weight.dtype)
        if bias is not None and n[2]:
            db = _C.colsum(d)[:V]
            if db.dtype != bias.dtype:
                db = db.to(bias.dtype)
        return dx, dw, db, None, None, None, None


def _head_wgrad(d, x2, V: int, tgt):
    """fp32 dW [V, K] = d[:, :V]ᵀ·x2, added into ``tgt`` when given (the
    existing W.grad) else returned: our split-M wgrad GEMM (pad rows dropped
    in its reduction pass) or hipBLASLt with an fp32 output (beta = 1 into
    ``tgt``), whichever the per-shape autotune measured faster — timed into a
    scratch target, so the measurement does not touch the gradient."""
    M, K = x2.shape
    Vp = d.shape[1]
    key = ("head_wgrad", M, Vp, K)

    def ours(t):
        return _C.conv1x1_wgrad(d, x2, accumulate_into=t, out_rows=V)

    def blas(t):
        if t is None:
            return torch.mm(d[:, :V].t(), x2, out_dtype=torch.float32)
        return torch.addmm(t, d[:, :V].t(), x2, out_dtype=torch.float32, out=t)

    impl = {"ring": ours, "hipblaslt": blas}
    c = _lin._CHOICE.get(key)
    if c is None:
        if _lin._AUTOTUNE and not torch.cuda.is_current_stream_capturing():
            scratch = torch.zeros(V, K, device=d.device, dtype=torch.float32)
            c = _pick(key, {name: (lambda f=f: f(scratch)) for name, f in impl.items()})
            del scratch
        else:
            c = "ring"
    return impl[c](tgt)


def lm_head_cross_entropy(x: torch.Tensor, weight: torch.Tensor, bias, target: torch.Tensor,
                          ignore_index: int = -100) -> torch.Tensor:
    """Mean cross-entropy of ``x @ weight.T (+ bias)`` against ``target``
    (``F.cross_entropy`` semantics, ``reduction="mean"``). Runs
    :class:`_LMHeadXentFn` for bf16 compute (bf16 ``x`` or bf16 autocast) when
    the model's LinearWeightPrep holds a current padded bf16 copy of
    ``weight`` (see ``padded_vocab``); otherwise the ATen GEMM +
    ``fused_cross_entropy``."""
    K = weight.shape[1]
    bf16 = x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                         and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    v = prepped_linear((weight,)) if x.is_cuda and bf16 else None
    if v is not None and K % 64 == 0 and x.numel() > 0 and v[0].shape[0] % 64 == 0:
        with torch.autocast("cuda", enabled=False):
            return _LMHeadXentFn.apply(x, weight, bias, target, v[0], v[1], ignore_index)
    logits = F.linear(x, weight, bias)
    flat = logits.reshape(-1, logits.shape[-1])
    return fused_cross_entropy(flat, target.reshape(-1), ignore_index=ignore_index) if x.is_cuda else \
        F.cross_entropy(flat.float(), target.reshape(-1), ignore_index=ignore_index)
