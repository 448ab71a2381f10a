"""Built-in DDP communication hooks (``DistributedDataParallel.register_comm_hook``).

Parity: torch's ``ddp_comm_hooks.default_hooks`` (allreduce / fp16 / bf16
compression). The default path (no hook) already averages in RCCL; for bf16
wire compression prefer ``DistributedDataParallel(..., comm_dtype=torch.bfloat16)``,
which fuses the cast into the pack launch. These hooks exist for API parity
and for experiments (``noop_hook`` measures compute-only step time).
"""
from __future__ import annotations

import torch

from .. import distributed as dist


def allreduce_hook(process_group, bucket):
    pg = process_group if process_group is not None else dist.get_default_group()
    buf = bucket.buffer()
    return pg.comm_for(buf).all_reduce(buf, dist.ReduceOp.AVG)


def _compress_hook(dtype):
    def hook(process_group, bucket):
        pg = process_group if process_group is not None else dist.get_default_group()
        buf = bucket.buffer()
        wire = buf.to(dtype)
        w = pg.comm_for(wire).all_reduce(wire, dist.ReduceOp.AVG)
        w.wait()
        buf.copy_(wire)
        return None

    return hook


fp16_compress_hook = _compress_hook(torch.float16)
bf16_compress_hook = _compress_hook(torch.bfloat16)


def noop_hook(process_group, bucket):
    """Skip communication entirely (benchmarking only: gradients stay local)."""
    return None
