"""On-device evaluation accumulator (fused arg-max / correct / NLL kernel).

    m = EvalMetrics(device, log_probs=True)
    for x, y in loader: m.update(model(x), y)      # no host sync per batch
    avg_loss, acc, n = m.compute(process_group)    # one all-reduce + one sync
"""
from __future__ import annotations

import torch

from .._ext import C as _C


class EvalMetrics:
    def __init__(self, device, log_probs: bool = False, ignore_index: int = -100):
        self.acc = torch.zeros(3, dtype=torch.float64, device=device)
        self.log_probs = log_probs
        self.ignore_index = ignore_index

    def reset(self):
        self.acc.zero_()

    @torch.no_grad()
    def update(self, scores: torch.Tensor, target: torch.Tensor):
        _C.eval_metrics_(self.acc, scores.reshape(-1, scores.shape[-1]), target.reshape(-1), self.log_probs,
                         self.ignore_index)

    def compute(self, group=None, all_reduce: bool = True):
        t = self.acc.clone()
        if all_reduce:
            from .. import distributed as dist

            if dist.is_initialized():
                dist.all_reduce(t, dist.ReduceOp.SUM, group=group)
        loss_sum, correct, n = t.tolist()
        return loss_sum / max(n, 1.0), correct / max(n, 1.0), int(n)
