"""1x1 convolutions on NHWC bf16 activations as hand-written MFMA GEMMs
(``csrc/kernels/gemm.hip``), fused with the neighbouring BatchNorm passes.

* :func:`conv1x1` — ``y = conv1x1(x, w)``; optionally also returns the
  per-output-channel (Σy, Σy²) accumulated in the GEMM epilogue, which the
  following :class:`~.batchnorm.BatchNormAct2d` consumes instead of running
  its own statistics pass over ``y``.
* :func:`bn_relu_conv1x1` — ``z = conv1x1(relu(bn(x)), w)`` in training mode:
  BN statistics of ``x`` (one read), then the GEMM applies BN + ReLU to ``x``
  while staging it into LDS — BN's output is never written to HBM. Backward:
  dgrad GEMM → BN+ReLU backward (mask recomputed from ``x``), and a wgrad
  GEMM that re-applies BN + ReLU to ``x`` in its prologue.

Weight gradients are produced in fp32 directly (no bf16→fp32 cast pass).
These replace MIOpen's 1x1 convolution kernels + the BN statistics/apply
kernels for ResNet-50's bottleneck 1x1 layers (the
reference framework's cuDNN/cuBLAS role).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .._ext import C as _C


def _cl(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()


# conv weight -> (bf16 [R,kh,kw,Cin], bf16 [Cin,kh,kw,R] tap-flipped) produced by
# the model's ConvWeightPrep for the forward in flight (one launch for every
# conv instead of one cast launch each); empty outside such a forward.
_PREPPED = {}


class ConvWeightPrep:
    """bf16 GEMM operands of a set of conv weights, all written by ONE kernel
    launch per forward (``weight_prep_kernel``) into a persistent flat buffer.

    ``with prep:`` runs the launch and publishes the views to the conv ops of
    this module for the duration of the forward; the backward keeps its own
    references (saved tensors) to the same persistent buffer, which the next
    forward rewrites only after the optimizer changed the weights. Rebuilt
    when a weight's storage moves. Capture-safe: fixed addresses, the launch is
    part of the captured forward."""

    def __init__(self, weights):
        self.weights = list(weights)
        self._key = None

    def __enter__(self):
        key = tuple(w.data_ptr() for w in self.weights)
        if key != self._key:
            self.table, self.tiles, self.wb, self.wt = _C.weight_prep_plan([w.detach() for w in self.weights])
            self._key = key
        _C.weight_prep_run(self.table, self.tiles)
        for w, b, t in zip(self.weights, self.wb, self.wt):
            _PREPPED[w] = (b, t)
        return self

    def __exit__(self, *exc):
        _PREPPED.clear()
        return False

    @staticmethod
    def eligible(w: torch.Tensor) -> bool:
        return (w.is_cuda and w.dtype == torch.float32 and w.dim() == 4
                and w.permute(0, 2, 3, 1).is_contiguous())


def _prepped(weight: torch.Tensor):
    return _PREPPED.get(weight) if _PREPPED else None


def _w2d(weight: torch.Tensor):
    """(bf16 [Cout, Cin], bf16 [Cin, Cout]): forward and dgrad B operands, one launch
    (none when the model's ConvWeightPrep already produced them this forward)."""
    p = _prepped(weight)
    if p is not None:
        b, t = p
        return b.view(b.shape[0], -1), t.view(t.shape[0], -1)
    return _C.weight_bf16_t(weight)


def gemm_ok(x: torch.Tensor, cin: int, cout: int) -> bool:
    """True when the MFMA 1x1 path handles this activation."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last)
            and bool(_C.conv1x1_supported(x.numel() // max(cin, 1), cout, cin)))


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stats):
        w, wt = _w2d(weight)
        y, st = _C.conv1x1_fwd(x, w, None, None, False, bool(stats))
        ctx.save_for_backward(x, wt)
        ctx.wshape, ctx.wdtype = weight.shape, weight.dtype
        ctx.mark_non_differentiable(st)
        ctx.set_materialize_grads(False)  # no zero-filled grad for the sums output
        return y, st

    @staticmethod
    def backward(ctx, gy, _gst):
        x, wt = ctx.saved_tensors
        if gy is None:
            return None, None, None
        gy = _cl(gy)
        dx = _C.conv1x1_dgrad(gy, wt) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = _C.conv1x1_wgrad(gy, x).view(ctx.wshape)
            if dw.dtype != ctx.wdtype:
                dw = dw.to(ctx.wdtype)
        return dx, dw, None


# BN-prologue 1x1 conv (ResNet layer-1 conv3): BN backward reduce in the dgrad
# epilogue (+0.6 %, profiles/r2_ab_pro_red.jsonl; False = separate reduce pass)
_PRO_RED = True


class _BNReluConv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, weight, running_mean, running_var, nbt, momentum, eps, stats, sums):
        # sums: (Σx, Σx²) of x from its producer's epilogue (no statistics pass)
        mean, invstd, scale, shift = _C.bn_stats_coef(x, gamma, beta, running_mean, running_var, float(momentum),
                                                      float(eps), nbt, sums)
        w, wt = _w2d(weight)
        z, st = _C.conv1x1_fwd(x, w, scale, shift, True, bool(stats))
        ctx.save_for_backward(x, gamma, beta, wt, mean, invstd, scale, shift)
        ctx.wshape, ctx.wdtype = weight.shape, weight.dtype
        ctx.mark_non_differentiable(st)
        ctx.set_materialize_grads(False)
        return z, st

    @staticmethod
    def backward(ctx, gz, _gst):
        x, gamma, beta, wt, mean, invstd, scale, shift = ctx.saved_tensors
        if gz is None:
            return (None,) * 11
        gz = _cl(gz)
        dw = _C.conv1x1_wgrad(gz, x, scale, shift, True).view(ctx.wshape)
        if dw.dtype != ctx.wdtype:
            dw = dw.to(ctx.wdtype)
        if _PRO_RED:
            # BN+ReLU backward reduction in the data-gradient GEMM's epilogue
            # (gemm.hip RED: mask recomputed from x), then the apply pass alone
            da, acc = _C.conv1x1_dgrad_bnred(gz, wt, x, gamma, beta, mean, invstd)
            dx, dgamma, dbeta = _C.bn_act_bwd_apply(da, x, gamma, beta, mean, invstd, acc)
        else:
            da = _C.conv1x1_dgrad(gz, wt)
            # BN + ReLU backward; the ReLU mask is recomputed from x (training coefficients)
            dx, dgamma, dbeta, _ = _C.bn_act_bwd(da, None, x, gamma, beta, mean, invstd, x, True, False, True, None)
        return dx, dgamma, dbeta, dw, None, None, None, None, None, None, None


def conv1x1(x: torch.Tensor, weight: torch.Tensor, stats: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """NHWC bf16 1x1 stride-1 convolution (no bias). Returns (y, sums) with
    ``sums`` = fp32 [2*Cout] (Σy, Σy²) when ``stats`` else an empty tensor."""
    return _Conv1x1Fn.apply(x, weight, stats)


def bn_relu_conv1x1(x: torch.Tensor, bn, weight: torch.Tensor, stats: bool = False,
                    sums: Optional[torch.Tensor] = None):
    """``conv1x1(relu(bn(x)), weight)`` for a training-mode ``BatchNorm2d``
    ``bn`` (its running statistics and ``num_batches_tracked`` are updated).
    ``sums``: x's (Σx, Σx²) from the producing kernel's epilogue, if any."""
    nbt = bn.num_batches_tracked
    if nbt is not None and (nbt.device != x.device or nbt.dtype != torch.int64):
        nbt.add_(1)
        nbt = None
    return _BNReluConv1x1Fn.apply(x, bn.weight, bn.bias, weight, bn.running_mean, bn.running_var, nbt, bn.momentum,
                                  bn.eps, stats, sums)


# downsample blocks: BN3's and the downsample BN's apply passes as one kernel
# (g read once; +0.95 %, profiles/r2_ab_bn_apply2.jsonl)
_APPLY2 = True
# identity block boundaries: BN3 + residual + ReLU as the A prologue of the next
# conv1 GEMM, which also stores y and its mask (gemm.hip RES) instead of a
# separate apply pass whose output the GEMM then re-reads. Correct (bit-identical
# y, test_gpu_fusions.py::test_res_prologue_matches_apply_pass) but measured
# SLOWER: ResNet-50 38.7 vs 36.2 ms per step (profiles/r4_res_prologue_ab.jsonl) —
# the prologue forces the BK = 32 BN-prologue ring on GEMMs that otherwise run
# the pipelined BK = 64 one, which costs more than the pass it removes (NOTES §25)
RES_PROLOGUE = False


class _BNResActConv1x1Fn(torch.autograd.Function):
    """Block boundary of a bottleneck chain, training mode:
    ``y = relu(bn3(z3) + r)`` with ``r`` the identity or ``bn_d(x2)`` (the
    downsample BN folded in), and the NEXT block's ``z1 = conv1x1(y, w)``
    (+ its BN1 sums). Returns (y, z1, sums): ``y`` feeds the next block's
    residual / downsample branch, ``z1`` its BN1.

    Backward: the conv1 data-gradient GEMM's epilogue adds the residual
    branch's gradient of ``y``, applies BN3's ReLU bits and reduces BN3's
    (and the downsample BN's) backward sums (gemm.hip RESRED) — it writes the
    masked gradient g, which is also the identity's gradient; BN3's separate
    reduce pass over (dy, dy2, z3) disappears and one apply pass per BN
    remains. Reference parity: the plain ``bn3 → add → relu → conv1``
    composition (``/root/reference/main.py`` trains through stock
    autograd)."""

    @staticmethod
    def forward(ctx, z3, gamma, beta, residual, x2, gamma2, beta2, w_next, rm, rv, nbt, stats, rm2, rv2, nbt2,
                stats2, momentum, eps, momentum2, eps2):
        ctx.set_materialize_grads(False)
        if x2 is not None:
            y, mean, invstd, bits, mean2, invstd2 = _C.bn_resbn_act_fwd(
                z3, gamma, beta, rm, rv, nbt, stats, x2, gamma2, beta2, rm2, rv2, nbt2, stats2, float(momentum),
                float(eps), float(momentum2), float(eps2))
            w, wt = _w2d(w_next)
            z1, s1 = _C.conv1x1_fwd(y, w, None, None, False, True)
        elif RES_PROLOGUE:
            # BN3 + residual + ReLU applied in conv1's A prologue; y and its mask
            # stored by the GEMM (no separate apply pass, no re-read of y)
            mean, invstd, scale, shift = _C.bn_stats_coef(z3, gamma, beta, rm, rv, float(momentum), float(eps), nbt,
                                                          stats)
            w, wt = _w2d(w_next)
            z1, s1, y, bits = _C.conv1x1_fwd_res(z3, w, scale, shift, _cl(residual), True)
            mean2 = invstd2 = None
        else:
            y, mean, invstd, bits = _C.bn_act_fwd(z3, gamma, beta, rm, rv, residual, True, float(momentum),
                                                  float(eps), True, nbt, stats)
            mean2 = invstd2 = None
            w, wt = _w2d(w_next)
            z1, s1 = _C.conv1x1_fwd(y, w, None, None, False, True)
        ctx.save_for_backward(z3, gamma, mean, invstd, bits, y, wt, x2, gamma2, mean2, invstd2)
        ctx.wshape, ctx.wdtype = w_next.shape, w_next.dtype
        ctx.mark_non_differentiable(s1)
        return y, z1, s1

    @staticmethod
    def backward(ctx, gy, gz, _gs):
        z3, gamma, mean, invstd, bits, y, wt, x2, gamma2, mean2, invstd2 = ctx.saved_tensors
        if gz is None:
            gz = torch.zeros((y.shape[0], ctx.wshape[0]) + tuple(y.shape[2:]), device=y.device, dtype=y.dtype)
        gz = _cl(gz)
        dw = _C.conv1x1_wgrad(gz, y)
        g, acc, acc2 = _C.conv1x1_dgrad_resred(gz, wt, z3, None if gy is None else _cl(gy), mean, bits, x2, mean2)
        dres = dx2 = dgamma2 = dbeta2 = None
        if x2 is not None and _APPLY2:  # both BNs' apply passes share one read of g
            dz3, dgamma, dbeta, dx2, dgamma2, dbeta2 = _C.bn_bwd_apply2_g(g, z3, gamma, mean, invstd, acc, x2, gamma2,
                                                                          mean2, invstd2, acc2)
        else:
            dz3, dgamma, dbeta = _C.bn_bwd_apply_g(g, z3, gamma, mean, invstd, acc)
            if x2 is not None:
                dx2, dgamma2, dbeta2 = _C.bn_bwd_apply_g(g, x2, gamma2, mean2, invstd2, acc2)
            else:
                dres = g  # relu mask already applied: the identity's gradient
        dw = dw.view(ctx.wshape)
        if dw.dtype != ctx.wdtype:
            dw = dw.to(ctx.wdtype)
        return (dz3, dgamma, dbeta, dres, dx2, dgamma2, dbeta2, dw) + (None,) * 12


def bn_res_act_conv1x1(bn3, z3: torch.Tensor, s3: torch.Tensor, identity: Optional[torch.Tensor], w_next,
                       resbn=None):
    """(y, z1, sums1) = (relu(bn3(z3) + identity-or-bn_d(x2)), conv1x1(y, w_next), Σ/Σ² of z1)
    for training-mode BatchNorms whose input sums come from their GEMM epilogues
    (``s3``; ``resbn`` = (bn_d, x2, s2)). Same parameters, buffers and running-
    statistic updates as the unfused composition."""

    def _nbt(m):
        t = m.num_batches_tracked
        if t is not None and (t.device != z3.device or t.dtype != torch.int64):
            t.add_(1)
            return None
        return t

    if resbn is not None:
        bn_d, x2, s2 = resbn
        return _BNResActConv1x1Fn.apply(z3, bn3.weight, bn3.bias, None, x2, bn_d.weight, bn_d.bias, w_next,
                                        bn3.running_mean, bn3.running_var, _nbt(bn3), s3, bn_d.running_mean,
                                        bn_d.running_var, _nbt(bn_d), s2, bn3.momentum, bn3.eps, bn_d.momentum,
                                        bn_d.eps)
    return _BNResActConv1x1Fn.apply(z3, bn3.weight, bn3.bias, identity, None, None, None, w_next, bn3.running_mean,
                                    bn3.running_var, _nbt(bn3), s3, None, None, None, None, bn3.momentum, bn3.eps,
                                    0.0, 0.0)


def res_conv_fuse_ok(bn3, z3: torch.Tensor, s3, next_conv) -> bool:
    """True when :func:`bn_res_act_conv1x1` handles BN3 ``bn3`` over ``z3`` feeding
    the 1x1 stride-1 conv ``next_conv``."""
    return (bn3.training and bn3.affine and bn3.track_running_stats and bn3.momentum is not None
            and s3 is not None and s3.numel() == 2 * z3.shape[1] and bn3.weight.dtype == torch.float32
            and next_conv.kernel_size == (1, 1) and next_conv.stride == (1, 1) and next_conv.bias is None
            and next_conv.groups == 1 and next_conv.in_channels == z3.shape[1]
            and next_conv.out_channels % 64 == 0 and next_conv.weight.dtype == torch.float32
            and gemm_ok(z3, next_conv.in_channels, next_conv.out_channels))


class _BNReluConvFn(torch.autograd.Function):
    """conv(relu(bn(x))) for a training-mode BatchNorm whose output is
    materialised (wide consumers, or gathered kxk convs where padding taps
    must stay zero): BN apply kernel (statistics from the producer's GEMM
    epilogue when given) → 1x1 GEMM or implicit-GEMM kxk conv (+ the next BN's
    sums). Backward: the data-gradient GEMM reduces the BN backward in its
    epilogue (gemm.hip RED), so BN's reduce pass over dy and x disappears;
    stride > 1 kxk falls back to MIOpen's data gradient + the full BN backward."""

    @staticmethod
    def forward(ctx, x, gamma, beta, weight, running_mean, running_var, nbt, momentum, eps, sums, k, stride, pad,
                stats):
        ctx.set_materialize_grads(False)
        y, mean, invstd, _ = _C.bn_act_fwd(x, gamma, beta, running_mean, running_var, None, True, float(momentum),
                                           float(eps), True, nbt, sums)
        if k == 1 and stride == 1:
            w, wt = _w2d(weight)
            z, st = _C.conv1x1_fwd(y, w, None, None, False, bool(stats))
        else:
            pre = _prepped(weight)
            if pre is not None:  # bf16 operands from the model's one-launch ConvWeightPrep
                wf, wt = pre     # wt: the flipped data-gradient weight [Cin][k][k][Cout]
                w = wf.permute(0, 3, 1, 2)
            else:
                w = weight.detach().to(torch.bfloat16)
                wf, wt = w.permute(0, 2, 3, 1).contiguous(), None
            z, st = _C.conv_fwd(y, wf, k, k, stride, pad, bool(stats))
        ctx.save_for_backward(x, y, gamma, beta, mean, invstd, w, wt)
        ctx.cfg = (k, stride, pad, weight.shape, weight.dtype)
        ctx.mark_non_differentiable(st)
        return z, st

    @staticmethod
    def backward(ctx, gz, _gst):
        if gz is None:
            return (None,) * 14
        x, y, gamma, beta, mean, invstd, w, wt = ctx.saved_tensors
        k, stride, pad, wshape, wdtype = ctx.cfg
        gz = _cl(gz)
        if k == 1 and stride == 1:
            dw = _C.conv1x1_wgrad(gz, y).view(wshape)
            dy, acc = _C.conv1x1_dgrad_bnred(gz, wt, x, gamma, beta, mean, invstd)
        else:
            dw = _C.conv_wgrad(gz, y, k, k, stride, pad)
            if stride == 1:
                wd = wt if wt is not None else w.flip(2, 3).permute(1, 2, 3, 0).contiguous()  # [Cin][k][k][Cout]
                dy, acc = _C.conv_dgrad_bnred(gz, wd, k, k, k - 1 - pad, x, gamma, beta, mean, invstd)
            else:
                dy = torch.ops.aten.convolution_backward(gz, y, w, None, [stride, stride], [pad, pad], [1, 1],
                                                         False, [0, 0], 1, [True, False, False])[0]
                dy = _cl(dy)
                acc = None
        if dw.dtype != wdtype:
            dw = dw.to(wdtype)
        if acc is None:
            dx, dgamma, dbeta, _ = _C.bn_act_bwd(dy, None, x, gamma, beta, mean, invstd, y, True, False, True, None)
        else:
            dx, dgamma, dbeta = _C.bn_act_bwd_apply(dy, x, gamma, beta, mean, invstd, acc)
        return dx, dgamma, dbeta, dw, None, None, None, None, None, None, None, None, None, None


def bn_relu_conv(x: torch.Tensor, bn, weight: torch.Tensor, k: int, stride: int, pad: int,
                 sums: Optional[torch.Tensor] = None, stats: bool = False):
    """``conv(relu(bn(x)), weight)`` (square k, no bias) for a training-mode
    BatchNorm ``bn`` on the MFMA kernels, BN backward reduced in the
    data-gradient GEMM's epilogue. Returns (z, sums of z when ``stats``)."""
    nbt = bn.num_batches_tracked
    if nbt is not None and (nbt.device != x.device or nbt.dtype != torch.int64):
        nbt.add_(1)
        nbt = None
    return _BNReluConvFn.apply(x, bn.weight, bn.bias, weight, bn.running_mean, bn.running_var, nbt, bn.momentum,
                               bn.eps, sums, k, stride, pad, stats)


class _ConvKxKFn(torch.autograd.Function):
    """kxk NHWC convolution: MIOpen forward and data gradient, our implicit-GEMM
    MFMA weight gradient (fp32 out; no zero-fill pass, no bf16→fp32 cast)."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding):
        w = weight.detach().to(torch.bfloat16)
        y = F.conv2d(x, w, None, stride, padding)
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.padding, ctx.wdtype = stride, padding, weight.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = _cl(gy)
        s, p = ctx.stride, ctx.padding
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(gy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        dw = None
        if ctx.needs_input_grad[1]:
            dw = _C.conv_wgrad(gy, x, w.shape[2], w.shape[3], s, p)
            if dw.dtype != ctx.wdtype:
                dw = dw.to(ctx.wdtype)
        return dx, dw, None, None


def conv_kxk(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> torch.Tensor:
    """NHWC bf16 kxk convolution (no bias, square stride/padding) whose weight
    gradient runs on the gathered MFMA wgrad kernel."""
    return _ConvKxKFn.apply(x, weight, stride, padding)


# stride-2 3x3 data gradient: the four parity classes of dx as ONE implicit-GEMM
# launch (conv_dgrad_s2_multi; four separate launches measured −0.4 % in the
# step, NOTES §19 — `_C.conv_dgrad_s2` stays as the op-level reference)


def _s2_tap_perm(wd: torch.Tensor) -> torch.Tensor:
    """The flipped data-gradient weight wd [Cin][3][3][Cout] as [Cin][9][Cout]
    with its taps in parity-class order 4 | 3 5 | 1 7 | 0 2 6 8 (classes
    (ph, pw) = 00, 01, 10, 11; see :func:`_parity_weights`): one cat of strided
    views (no index tensor, capture-safe)."""
    w9 = wd.reshape(wd.shape[0], 9, wd.shape[3])
    return torch.cat([w9[:, 4:5], w9[:, 3:6:2], w9[:, 1:8:6], w9[:, 0:3:2], w9[:, 6:9:2]], dim=1)


def _parity_weights(wd: torch.Tensor):
    """bf16 [Cin][nkh][nkw][Cout] weight subsets of a 3x3 / stride-2 / pad-1
    conv for dx parity classes (ph, pw) = 00, 01, 10, 11, as strided views of
    the flipped data-gradient weight wd [Cin][3][3][Cout] (wd[.., kh', ..] =
    w[.., 2-kh', ..]): dx row 2a+ph takes kernel rows kh ≡ ph+1 (mod 2) from gy
    rows a + (ph+1-kh)/2, ordered by that offset (even: kh 1 → +0; odd: kh 2 →
    +0, kh 0 → +1, i.e. kh' = 0, 2). No index tensors (list indexing copies
    them host→device and stalls the launch stream)."""
    sl = (slice(1, 2), slice(0, 3, 2))
    return [wd[:, sl[ph], sl[pw], :].contiguous() for ph in (0, 1) for pw in (0, 1)]


class _ConvKxKGemmFn(torch.autograd.Function):
    """kxk NHWC convolution on the implicit-GEMM MFMA kernels (gemm.hip
    GATHER): forward (+ the next BatchNorm's Σy, Σy² from the epilogue), data
    gradient for stride 1 as the forward kernel on gy with the flipped,
    transposed weight, for stride 2 the parity-class launch (3x3) or the
    scattering GEMM (1x1), weight gradient on the gathered wgrad kernel."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, stats):
        ctx.set_materialize_grads(False)
        pre = _prepped(weight)
        if pre is not None:  # operands from the model's one-launch ConvWeightPrep
            wf, wd = pre
            w = wf.permute(0, 3, 1, 2)  # channels_last bf16 [Cout, Cin, kh, kw] view
        else:
            w = weight.detach().to(torch.bfloat16)
            wf = wd = None
        kh, kw = w.shape[2], w.shape[3]
        if wf is None:
            # both bf16 operands (forward, flipped data-gradient) from one cast launch
            wf, wd = _C.conv_weight_bf16(weight) if kh == kw else (w.permute(0, 2, 3, 1).contiguous(), None)
        y, st = _C.conv_fwd(x, wf, kh, kw, stride, padding, stats)
        ctx.save_for_backward(x, w, wd)
        ctx.cfg = (stride, padding, weight.dtype)
        ctx.mark_non_differentiable(st)
        return y, st

    @staticmethod
    def backward(ctx, gy, _gst=None):
        x, w, wd = ctx.saved_tensors
        s, p, wdtype = ctx.cfg
        gy = _cl(gy)
        kh, kw = w.shape[2], w.shape[3]
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = _C.conv_wgrad(gy, x, kh, kw, s, p)
        if ctx.needs_input_grad[0]:
            if s == 1 and kh - 1 - p >= 0 and kw == kh:
                if wd is None:
                    wd = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()  # [Cin][kh][kw][Cout]
                dx = _C.conv_fwd(gy, wd, kh, kw, 1, kh - 1 - p, False)[0]
            elif (kh == kw == 1 and s == 2 and p == 0 and wd is not None and x.shape[2] == 2 * gy.shape[2]
                  and x.shape[3] == 2 * gy.shape[3]):
                # strided 1x1 (downsample): GEMM whose epilogue scatters to the even pixels, zeros the rest
                dx = _C.conv1x1_s2_dgrad(gy, wd)
            elif (kh == kw == 3 and s == 2 and p == 1 and x.shape[1] % 64 == 0
                  and (x.shape[2] + 1) // 2 == gy.shape[2] and (x.shape[3] + 1) // 2 == gy.shape[3]):
                if wd is None:
                    wd = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
                dx = _C.conv_dgrad_s2_multi(gy, _s2_tap_perm(wd), x.shape[2], x.shape[3])
            else:
                dx = torch.ops.aten.convolution_backward(gy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                         [True, False, False])[0]
        if dw is not None and dw.dtype != wdtype:
            dw = dw.to(wdtype)
        return dx, dw, None, None, None


def conv_kxk_gemm(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int, stats: bool = False):
    """NHWC bf16 kxk convolution on the implicit-GEMM MFMA kernels. Returns
    (y, sums) — sums = fp32 [2*Cout] (Σy, Σy²) when ``stats`` else empty.
    (Round 1 kept a per-shape MIOpen routing policy; our forward + BN sums
    and our gathered wgrad measured faster than MIOpen at every ResNet-50
    shape, profiles/r1_gemm3x3_bk64.log, r1_gemm_bench_wgrad_bk64.log.)"""
    return _ConvKxKGemmFn.apply(x, weight, stride, padding, stats)


def conv_kxk_gemm_ok(x: torch.Tensor, conv) -> bool:
    return (conv_kxk_ok(x, conv) and x.shape[1] % 64 == 0 and conv.out_channels % 64 == 0
            and conv.kernel_size[0] == conv.kernel_size[1] and conv.kernel_size[0] <= 8)


def conv_kxk_ok(x: torch.Tensor, conv) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and conv.bias is None
            and conv.groups == 1 and conv.dilation == (1, 1)
            and x.is_contiguous(memory_format=torch.channels_last)
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0
            and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1])
