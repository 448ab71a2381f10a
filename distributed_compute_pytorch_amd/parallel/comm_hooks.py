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
        # cast to the wire dtype on the compute stream (the pack), average in
        # that dtype, cast back into the bucket on the collective's stream: the
        # returned Work completes after the cast back, and nothing waits here
        # (the Reducer's finalize orders the consumers after it)
        pg = process_group if process_group is not None else dist.get_default_group()
        buf = bucket.buffer()
        wire = buf.to(dtype)
        return pg.comm_for(wire).all_reduce_into(wire, buf, dist.ReduceOp.AVG)

    hook.wire_dtype = dtype
    return hook


fp16_compress_hook = _compress_hook(torch.float16)
bf16_compress_hook = _compress_hook(torch.bfloat16)


def noop_hook(process_group, bucket):
    """Skip communication entirely (benchmarking only: gradients stay local)."""
    return None


class ContentionEmulation:
    """State of :func:`contention_emulation_hook`: the emulated job has
    ``world`` ranks whose ring all-reduce reaches ``busbw_gbps`` bus bandwidth
    over xGMI with ``channels`` RCCL channels (one workgroup each) and a
    per-collective latency of ``alpha_us``."""

    def __init__(self, world: int = 8, busbw_gbps: float = 300.0, channels: int = 16, alpha_us: float = 20.0,
                 process_group=None):
        self.world, self.busbw_gbps, self.channels, self.alpha_us = world, busbw_gbps, channels, alpha_us
        self.process_group = process_group


def contention_emulation_hook(state: ContentionEmulation, bucket):
    """One-GPU stand-in for an N-rank bucket all-reduce (NOTES §22): on the
    collective stream, ``state.channels`` workgroups move the ring
    all-reduce's 2(N-1)/N × bucket bytes through HBM and hold their CUs for
    the collective's modelled duration, so the backward GEMMs / BN kernels
    share the chip with it exactly when the real collective would run. The
    bucket's (1-rank, already averaged) gradient is left untouched; the
    returned Work orders finalize after the emulated collective. Needs the
    RCCL communicator's comm-stream path (``DCP_SINGLE_RANK_HOP=1`` at one
    rank)."""
    pg = state.process_group if state.process_group is not None else dist.get_default_group()
    buf = bucket.buffer()
    return pg.comm_for(buf).emulate_all_reduce(buf, state.world, state.busbw_gbps, state.channels, state.alpha_us)
