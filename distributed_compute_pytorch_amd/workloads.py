"""Training workloads for the BASELINE.json configs (used by bench.py and the
examples): model + optimizer + synthetic data + one training step.

Configs (BASELINE.json):
  #1 mlp       2-layer MLP on MNIST-shaped synthetic tensors (CPU/host backend ok)
  #2 resnet50  ResNet-50 DDP bf16, synthetic ImageNet 224×224 (headline)
  #3 bert      BERT-base pre-training (MLM+NSP) DDP bf16, seq 512
  #4 resnet50  bucket-size sweep (bench.py --bucket-cap-mb)
  #5 gpt2      GPT-2-small DDP + gradient accumulation (no_sync) + bf16 AMP, seq 1024
  (+) convnet  the reference MNIST ConvNet with Adadelta (main.py)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.nn.functional as F

from . import optim as dopt
from .utils.data import SyntheticBatches


@dataclass
class Workload:
    name: str
    model: torch.nn.Module
    data: object
    make_optimizer: Callable
    loss_fn: Callable
    per_gpu_batch: int
    seq_len: Optional[int]
    accum: int = 1
    amp: bool = True
    channels_last: bool = False
    sample_unit: str = "samples"


class _BertData:
    def __init__(self, batch, seq, device, preds=80, pool=2, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.batches = []
        for _ in range(pool):
            ids = torch.randint(0, 30522, (batch, seq), generator=g)
            pos = torch.stack([torch.randperm(seq, generator=g)[:preds].sort().values for _ in range(batch)])
            lab = torch.randint(0, 30522, (batch, preds), generator=g)
            nsp = torch.randint(0, 2, (batch,), generator=g)
            tt = (torch.arange(seq)[None, :] >= seq // 2).long().expand(batch, seq).contiguous()
            self.batches.append(tuple(t.to(device) for t in (ids, tt, pos, lab, nsp)))
        self.i = 0

    def __next__(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


class _TokenData:
    def __init__(self, batch, seq, vocab, device, pool=2, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.batches = []
        for _ in range(pool):
            t = torch.randint(0, vocab, (batch, seq + 1), generator=g)
            self.batches.append((t[:, :-1].contiguous().to(device), t[:, 1:].contiguous().to(device)))
        self.i = 0

    def __next__(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


def build(name: str, device, batch: Optional[int] = None, fused: bool = True, seq_len: Optional[int] = None,
          accum: Optional[int] = None, channels_last: bool = True, fused_gemm: Optional[bool] = None) -> Workload:
    from . import models

    name = name.lower()
    if name == "resnet50":
        # 1024 per GPU (41 GiB peak of the 288 GB HBM): +4 % over 512 on one
        # MI355X (the per-step fixed costs — optimizer, weight prep, tails of
        # the persistent grids — amortised over twice the images, layer 3/4
        # tiles filling more rounds; stock torch gains 3.7 %) and half the
        # all-reduce bytes per sample at N > 1 again
        # (profiles/r6_resnet_batch_sweep.jsonl: 512 / 768 / 1024 / 2048 =
        # 14,033 / 14,414 / 14,629 / 15,088; round 1 chose 512 over 256,
        # profiles/r1_resnet50_b512_pairs79.jsonl)
        b = batch or 1024
        m = models.resnet50(fused_bn=fused, fused_gemm=fused if fused_gemm is None else (fused and fused_gemm)).to(device)
        if channels_last:
            m = m.to(memory_format=torch.channels_last)
        data = SyntheticBatches(b, (3, 224, 224), 1000, device, channels_last=channels_last, pool=2)
        return Workload(name, m, data,
                        lambda params: dopt.SGD(params, lr=0.1, momentum=0.9, weight_decay=1e-4),
                        lambda model, batch_: F.cross_entropy(model(batch_[0]), batch_[1]), b, None,
                        channels_last=channels_last)
    if name == "gpt2":
        b = batch or 8
        T = seq_len or 1024
        m = models.gpt2_small(fused=fused).to(device)
        data = _TokenData(b, T, 50257, device)
        return Workload(name, m, data,
                        lambda params: dopt.AdamW(params, lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1),
                        lambda model, batch_: model(batch_[0], batch_[1]), b, T, accum=accum or 4)
    if name == "bert":
        b = batch or 32
        T = seq_len or 512
        m = models.bert_base(fused=fused).to(device)
        data = _BertData(b, T, device, preds=max(1, int(round(T * 0.15625))))
        return Workload(name, m, data,
                        lambda params: dopt.AdamW(params, lr=1e-4, weight_decay=0.01),
                        lambda model, bt: model(bt[0], token_type_ids=bt[1], mlm_positions=bt[2], mlm_labels=bt[3],
                                                nsp_labels=bt[4]), b, T, accum=accum or 1)
    if name == "convnet":
        b = batch or 128
        m = models.ConvNet(fused=fused and device.type == "cuda").to(device)
        data = SyntheticBatches(b, (1, 28, 28), 10, device, pool=4)
        return Workload(name, m, data, lambda params: dopt.Adadelta(params, lr=1e-3),
                        lambda model, bt: F.nll_loss(model(bt[0]), bt[1]), b, None, amp=False)
    if name == "mlp":
        b = batch or 128
        m = models.MLP().to(device)
        data = SyntheticBatches(b, (1, 28, 28), 10, device, pool=4)
        return Workload(name, m, data, lambda params: dopt.Adadelta(params, lr=1e-3),
                        lambda model, bt: F.nll_loss(model(bt[0]), bt[1]), b, None, amp=False)
    raise ValueError(f"unknown workload {name!r}")


def make_step(wl: Workload, ddp, opt, device_type: str = "cuda", graph: bool = False, set_to_none: bool = True):
    """One optimizer step = ``accum`` micro-batches (all but the last under
    ``no_sync``), bf16 autocast when ``wl.amp``. ``graph=True`` captures the
    whole step (fwd + bwd + reduction + optimizer) into one HIP graph and
    replays it (see :mod:`.utils.graphs`). ``set_to_none=False`` zeroes the
    gradients in place instead (they stay the DDP bucket views, so the
    backward's kernels accumulate straight into them)."""

    def run(*flat):
        opt.zero_grad(set_to_none=set_to_none)
        loss = None
        n = len(flat) // wl.accum
        for k in range(wl.accum):
            batch = flat[k * n:(k + 1) * n]
            ctx = ddp.no_sync() if (k < wl.accum - 1 and hasattr(ddp, "no_sync")) else _Null()
            with ctx:
                with torch.autocast(device_type, dtype=torch.bfloat16, enabled=wl.amp):
                    loss = wl.loss_fn(ddp, batch)
                    if wl.accum > 1:
                        loss = loss / wl.accum
                loss.backward()
        opt.step()
        return loss

    def next_flat():
        out = []
        for _ in range(wl.accum):
            out.extend(next(wl.data))
        return out

    if not graph:
        return lambda: run(*next_flat())
    from .utils.graphs import CapturedStep, capture_stream

    for g in opt.param_groups:  # Adam/AdamW: device-side step (bias corrections advance on replay)
        if "capturable" in g:
            g["capturable"] = True

    static = [t.clone() for t in next_flat()]
    captured = CapturedStep(run, static, stream=capture_stream())
    return lambda: captured(*next_flat())


def pretune_step(wl: Workload, ddp, opt, device_type: str = "cuda") -> bool:
    """One untimed micro-step under ``no_sync`` inside :class:`ops.linear.pretune`
    (transformer workloads): every Linear / LM-head GEMM shape is autotuned
    with no bucket collective in flight, and rank 0's table is adopted by all
    ranks in one store round. The gradients it produced are dropped. False
    (nothing run) when the model has no autotuned GEMMs or no ``no_sync``."""
    from .ops import linear as _lin

    if not (_lin._AUTOTUNE and hasattr(ddp, "no_sync")
            and any(isinstance(m, _lin.FusedLinear) for m in wl.model.modules())):
        return False
    batch = list(next(wl.data))
    with _lin.pretune(), ddp.no_sync():
        with torch.autocast(device_type, dtype=torch.bfloat16, enabled=wl.amp):
            loss = wl.loss_fn(ddp, batch)
        loss.backward()
    _lin.discard_weight_grads()
    opt.zero_grad(set_to_none=True)
    for p in wl.model.parameters():
        p.grad = None
    return True


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
