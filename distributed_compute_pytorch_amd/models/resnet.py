"""ResNet-50 (v1.5: stride on the 3×3 conv) — BASELINE configs #2 and #4.

Architecture and init follow the standard ImageNet ResNet-50 (25,557,032
parameters; kaiming-normal fan_out convs, BN γ=1/β=0, optional zero-init of
the last BN γ in each residual branch). Written from scratch (torchvision is
not available here).

MI355X layout: the model is meant to run channels_last (NHWC) in bf16
autocast — MIOpen's NHWC implicit-GEMM convolutions feed the MFMA cores
without layout transposes. ``fused_bn=True`` replaces every BN(+ReLU)(+residual
add) with the hand-written HIP kernels of :mod:`..ops.batchnorm` (one read +
one write per activation in the forward, statistics fused).
"""
from __future__ import annotations

from typing import List, Optional, Type

import torch
from torch import nn

from ..ops.batchnorm import BatchNormAct2d, bn_resbn_act, resbn_ok
from ..ops.conv import (ConvWeightPrep, bn_relu_conv, bn_relu_conv1x1, bn_res_act_conv1x1, conv1x1 as gemm_conv1x1,
                        conv_kxk_gemm, conv_kxk_gemm_ok, gemm_ok, res_conv_fuse_ok)
from ..ops.pool import FusedMaxPool2d, global_avg_pool_flat
from ..ops.stem import fused_stem, stem_supported


# Fusion table of the fused ResNet path (plain constants, no environment
# switches: the A/B history of each entry is in NOTES.md / profiles/; tests
# monkeypatch them to check every fused path against the unfused one).
#
# BN1→conv2 / BN2→conv3 as one autograd node whose data-gradient GEMM reduces
# the BN backward in its epilogue (gemm.hip RED). Bit mask: 1 = BN1→conv2
# (stride-1 3x3 on the gathered GEMM, Cin > 64), 2 = BN2→conv3 (1x1, the wide
# layers whose BN2 is not a GEMM prologue), 4 = BN1→conv2 for Cin = 64 (layer 1:
# the direct 3x3 kernel's RED epilogue): +0.55 % / +0.3 % / +0.27 %
# (profiles/r2_ab_bn_conv_fuse7.jsonl, r2_ab_bn_conv_fuse.jsonl, r2_ab_bn1_red_c64.jsonl).
BN_CONV_FUSE = 7
# BN-apply prologue in the conv3 GEMM only while Cout ≤ this (≤ 2 N-tiles of
# 128; 512 measured neutral, profiles/r2_ab_pro_max_cout.jsonl)
PRO_MAX_COUT = 256
# conv1 + bn1 + relu + maxpool as one fused node (ops/stem.py); False = per-module path
FUSED_STEM = True
# every bottleneck conv's bf16 operands from ONE launch per forward (ops/conv.py ConvWeightPrep)
WEIGHT_PREP = True
# downsample BN applied inside BN3's residual kernel (its output never written)
RESBN = True
# each block's BN3 + residual + ReLU and the NEXT block's conv1 as one autograd
# node: BN3's backward reduction runs in conv1's data-gradient epilogue
RES_CONV_FUSE = True


def conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride, 1, bias=False)


def conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride, 0, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 fused_bn: bool = False, fused_gemm: Optional[bool] = None):
        super().__init__()
        # 1x1 convs as MFMA GEMMs fused with the BN passes (training, bf16 NHWC)
        self.fused_gemm = fused_bn if fused_gemm is None else fused_gemm
        cout = width * self.expansion
        self.conv1 = conv1x1(cin, width)
        self.bn1 = BatchNormAct2d(width, act=True, fused=fused_bn)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = BatchNormAct2d(width, act=True, fused=fused_bn)
        self.conv3 = conv1x1(width, cout)
        # BN3 + residual add + ReLU are one fused op
        self.bn3 = BatchNormAct2d(cout, act=True, residual=True, fused=fused_bn)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor, identity: Optional[torch.Tensor] = None, dual: bool = False):
        """``identity``: alias of ``x`` produced by the previous block's
        dual-output BN (its gradient is summed inside that BN's backward);
        it feeds the residual add, or the downsample branch when there is one."""
        if self._gemm_path(x):
            y, a, _ = self._forward_gemm(x, identity, dual)
            return (y, a) if dual else y
        if self.downsample is not None:
            identity = self.downsample(x if identity is None else identity)
        elif identity is None:
            identity = x
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        return self.bn3(self.conv3(out), identity, dual=dual)

    def chain(self, x, identity, head, nxt: Optional["Bottleneck"]):
        """One step of a chained bottleneck sequence: returns (y, alias, head).
        ``head`` = (z1, sums) of this block's conv1, already computed by the
        previous block's fused BN3→conv1 node (then ``x`` only feeds the
        residual / downsample branch); ``nxt`` = the following block (None
        for the last one). The returned ``head`` is set when this block
        fused its BN3 with ``nxt``'s conv1, else ``alias`` is the dual-output
        alias of ``y`` for ``nxt``'s residual (or None after the last block)."""
        if self._gemm_path(x):
            return self._forward_gemm(x, identity, nxt is not None, head, nxt)
        if head is not None:
            raise RuntimeError("chained conv1 output handed to a block off the fused GEMM path")
        if nxt is None:
            return self.forward(x, identity, dual=False), None, None
        y, a = self.forward(x, identity, dual=True)
        return y, a, None

    def _gemm_path(self, x: torch.Tensor) -> bool:
        if not (self.fused_gemm and self.training and self.bn1.fused and self.bn2.fused and self.bn3.fused):
            return False
        return (gemm_ok(x, self.conv1.in_channels, self.conv1.out_channels)
                and self.conv3.out_channels % 64 == 0 and self.conv3.in_channels % 64 == 0)

    def _forward_gemm(self, x, identity, dual, head=None, nxt=None):
        """conv1 (GEMM, BN1 sums in its epilogue) → BN1+ReLU apply → conv2
        (MIOpen 3x3) → BN2 statistics → conv3 GEMM with BN2+ReLU applied in its
        prologue and BN3 sums in its epilogue → BN3 + residual + ReLU apply.
        Per block this drops the BN1/BN3 statistics passes and BN2's apply
        (a full write + read of the 3x3 conv's activation). Returns (y, alias
        or None, next block's conv1 head or None) — see :meth:`chain`."""
        inp = x if identity is None else identity
        resbn = None  # (downsample BN, its raw input, its sums): applied inside BN3's kernel
        if self.downsample is not None:
            conv, bn = self.downsample[0], self.downsample[1]
            z = st = None
            if conv.stride == (1, 1) and gemm_ok(inp, conv.in_channels, conv.out_channels):
                z, st = gemm_conv1x1(inp, conv.weight, stats=True)
            elif conv_kxk_gemm_ok(inp, conv):
                # strided 1x1: gathered implicit GEMM (+ BN sums); dgrad on MIOpen
                z, st = conv_kxk_gemm(inp, conv.weight, conv.stride[0], conv.padding[0], stats=True)
            if z is None:
                identity = self.downsample(inp)
            elif RESBN and resbn_ok(bn, z, st) and resbn_ok(self.bn3, z, st):
                resbn, identity = (bn, z, st), None
            else:
                identity = bn(z, stats=st)
        else:
            identity = inp
        z1, s1 = head if head is not None else gemm_conv1x1(x, self.conv1.weight, stats=True)
        c2 = self.conv2
        s2 = None
        fuse3 = bool(BN_CONV_FUSE & 2)
        if (conv_kxk_gemm_ok(z1, c2) and c2.stride == (1, 1)
                and ((BN_CONV_FUSE & 1 and c2.in_channels > 64) or (BN_CONV_FUSE & 4 and c2.in_channels == 64))):
            x2, s2 = bn_relu_conv(z1, self.bn1, c2.weight, c2.kernel_size[0], c2.stride[0], c2.padding[0], sums=s1,
                                  stats=True)
            return self._tail(x2, s2, identity, dual, fuse3, resbn, nxt)
        y1 = self.bn1(z1, stats=s1)
        if conv_kxk_gemm_ok(y1, c2):
            x2, s2 = conv_kxk_gemm(y1, c2.weight, c2.stride[0], c2.padding[0], stats=True)
        else:
            x2 = c2(y1)
        if not x2.is_contiguous(memory_format=torch.channels_last):
            x2 = x2.contiguous(memory_format=torch.channels_last)
        return self._tail(x2, s2, identity, dual, fuse3, resbn, nxt)

    def _tail(self, x2, s2, identity, dual, fuse, resbn=None, nxt=None):
        """BN2 → conv3 → BN3 (+ residual, ReLU) [→ nxt's conv1]: (y, alias, head)."""
        if self.conv3.out_channels <= PRO_MAX_COUT:
            # BN2+ReLU applied in the GEMM prologue (its output never hits HBM)
            z3, s3 = bn_relu_conv1x1(x2, self.bn2, self.conv3.weight, stats=True, sums=s2)
        elif fuse:
            # BN2 output materialised once; BN2's backward reduce in conv3's dgrad epilogue
            z3, s3 = bn_relu_conv(x2, self.bn2, self.conv3.weight, 1, 1, 0, sums=s2, stats=True)
        else:
            # wide conv3: every N-tile re-applies the prologue to the same rows,
            # which costs more than one apply pass over the narrow input
            z3, s3 = gemm_conv1x1(self.bn2(x2, stats=s2), self.conv3.weight, stats=True)
        if (nxt is not None and RES_CONV_FUSE and res_conv_fuse_ok(self.bn3, z3, s3, nxt.conv1)
                and nxt._gemm_path(z3) and (resbn is None or resbn_ok(self.bn3, z3, s3))):
            y, z1, sums1 = bn_res_act_conv1x1(self.bn3, z3, s3, identity, nxt.conv1.weight, resbn)
            return y, None, (z1, sums1)
        if resbn is not None:
            if resbn_ok(self.bn3, z3, s3):
                bn, z, st = resbn
                out = bn_resbn_act(self.bn3, z3, s3, bn, z, st, dual)
                return (out[0], out[1], None) if dual else (out, None, None)
            identity = resbn[0](resbn[1], stats=resbn[2])
        out = self.bn3(z3, identity, dual=dual, stats=s3)
        return (out[0], out[1], None) if dual else (out, None, None)


class BottleneckStage(nn.Sequential):
    """nn.Sequential of bottlenecks (same state_dict keys) that threads the
    dual-output BN alias from each block into the next block's residual."""

    use_dual = True

    def forward(self, x, ident=None, dual_out: bool = False):
        """``ident``: alias of ``x`` from the previous stage's dual output;
        ``dual_out``: return (y, alias) from the last block as well (for the
        next stage's first block, whose conv1 and downsample both read y)."""
        blocks = list(self)
        for i, blk in enumerate(blocks):
            last = i + 1 == len(blocks)
            dual = self.use_dual and (dual_out if last else True)
            out = blk(x, ident, dual=dual)
            x, ident = (out if dual else (out, None))
        return (x, ident) if dual_out and self.use_dual else x


def _downsample(cin, cout, stride, fused_bn):
    # nn.Sequential keeps torchvision's state_dict keys (downsample.0 / downsample.1)
    return nn.Sequential(conv1x1(cin, cout, stride), BatchNormAct2d(cout, act=False, fused=fused_bn))


class ResNet(nn.Module):
    def __init__(self, block: Type[Bottleneck], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, fused_bn: bool = False, fused_pool: Optional[bool] = None,
                 dual_bn: bool = True, fused_gemm: Optional[bool] = None):
        super().__init__()
        self.inplanes = 64
        self.fused_bn = fused_bn
        self.fused_gemm = fused_bn if fused_gemm is None else fused_gemm
        self.dual_bn = dual_bn
        fused_pool = fused_bn if fused_pool is None else fused_pool
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = BatchNormAct2d(64, act=True, fused=fused_bn)
        self.maxpool = (FusedMaxPool2d if fused_pool else nn.MaxPool2d)(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, BatchNormAct2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _make_layer(self, block, width, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != width * block.expansion:
            downsample = _downsample(self.inplanes, width * block.expansion, stride, self.fused_bn)
        layers = [block(self.inplanes, width, stride, downsample, self.fused_bn, self.fused_gemm)]
        self.inplanes = width * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, width, fused_bn=self.fused_bn, fused_gemm=self.fused_gemm))
        stage = BottleneckStage(*layers)
        stage.use_dual = self.dual_bn
        return stage

    def _chain(self, x, a):
        """Every bottleneck of the four stages as one chain (block i's BN3 fused
        with block i+1's conv1 where both run on the GEMM path)."""
        blocks = [b for st in (self.layer1, self.layer2, self.layer3, self.layer4) for b in st]
        head = None
        for i, blk in enumerate(blocks):
            x, a, head = blk.chain(x, a, head, blocks[i + 1] if i + 1 < len(blocks) else None)
        return x

    def _weight_prep(self):
        """Context that casts every bottleneck conv weight to its bf16 GEMM
        operands in one launch (training on the fused GEMM path), else a no-op."""
        import contextlib

        if not (WEIGHT_PREP and self.fused_gemm and self.training and self.fc.weight.is_cuda):
            return contextlib.nullcontext()
        prep = self.__dict__.get("_wprep")
        if prep is None:
            ws = [m.weight for name, m in self.named_modules()
                  if isinstance(m, nn.Conv2d) and m is not self.conv1]
            if not ws or not all(ConvWeightPrep.eligible(w) for w in ws):
                return contextlib.nullcontext()
            prep = ConvWeightPrep(ws)
            self.__dict__["_wprep"] = prep  # not a submodule / buffer: state_dict unchanged
        return prep

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        with self._weight_prep():
            return self._forward(x)

    def _forward(self, x: torch.Tensor) -> torch.Tensor:
        if (FUSED_STEM and self.fused_bn and isinstance(self.maxpool, FusedMaxPool2d)
                and stem_supported(x, self.conv1, self.bn1, self.training)):
            # stem GEMM + BN + ReLU + max-pool in one node (no MIOpen, no ATen casts)
            if self.dual_bn and RES_CONV_FUSE:
                x = self._chain(*fused_stem(x, self.conv1, self.bn1, dual=True))
            elif self.dual_bn:
                x, a = fused_stem(x, self.conv1, self.bn1, dual=True)
                x, a = self.layer1(x, a, True)
                x, a = self.layer2(x, a, True)
                x, a = self.layer3(x, a, True)
                x = self.layer4(x, a, False)
            else:
                x = self.layer4(self.layer3(self.layer2(self.layer1(fused_stem(x, self.conv1, self.bn1)))))
            return self.fc(global_avg_pool_flat(x))
        x = self.bn1(self.conv1(x))
        if self.fused_bn and self.dual_bn:
            # thread dual-output aliases across stage boundaries: every
            # fan-out gradient is summed inside a BN / pool backward kernel
            if isinstance(self.maxpool, FusedMaxPool2d):
                x, a = self.maxpool(x, dual=True)
            else:
                x, a = self.maxpool(x), None
            if RES_CONV_FUSE:
                x = self._chain(x, a)
            else:
                x, a = self.layer1(x, a, True)
                x, a = self.layer2(x, a, True)
                x, a = self.layer3(x, a, True)
                x = self.layer4(x, a, False)
        else:
            x = self.layer4(self.layer3(self.layer2(self.layer1(self.maxpool(x)))))
        x = global_avg_pool_flat(x) if self.fused_bn else torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet18_like(num_classes: int = 10, **kw) -> ResNet:
    """Tiny bottleneck ResNet for tests (same code path, few layers)."""
    return ResNet(Bottleneck, [1, 1, 1, 1], num_classes, **kw)
