"""Whole-step HIP-graph capture (forward + backward + DDP reduction + optimizer).

On this box a ResNet-50 step issues ~800 kernels; the host needs ~35-45 ms
to issue them (MIOpen's per-call dispatch dominates) — as long as the GPU
needs to run them. Capturing the whole training step once and replaying it
makes the step GPU-bound ("HIP streams and graphs instead of a
tracing compiler"; task: "capture launch-bound inner loops in hipGraphs").

Everything the step touches is capture-safe by construction:
* the Reducer's pack launches, RCCL collectives (RCCL supports capture) and
  comm-stream event edges are recorded into the graph; the watchdog skips
  captured work;
* no memset / memcpy nodes: on this ROCm a captured hipMemsetAsync /
  hipMemcpyAsync node is not reliably ordered before the next kernel node on
  replays after the first (tools/graph_op_check.py), so zeroed accumulators
  come from fill kernels under capture and multi-tensor kernel tables are
  uploaded once, outside the graph, and kept alive for good;
* the fused optimizers read hyper-parameters at capture time — changing the
  LR after capture requires re-capturing (``CapturedStep.recapture``).

The autograd engine binds every parameter's AccumulateGrad node to the stream
that was current when the node was created, and the Reducer keeps those nodes
alive; so construct the DDP model (and run warmup / capture) under ONE side
stream — :func:`capture_stream` returns it::

    s = capture_stream()
    with torch.cuda.stream(s):
        ddp = DistributedDataParallel(model, ...)
        opt = SGD(ddp.parameters(), ...)
    step = CapturedStep(step_fn, static_batch, stream=s)   # step_fn(batch) -> loss
    for batch in loader:
        loss = step(batch)                                 # copies into static buffers, replays
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


_STREAMS = {}


def capture_stream(device=None) -> torch.cuda.Stream:
    """The per-device side stream used for DDP construction, warmup and capture."""
    dev = torch.cuda.current_device() if device is None else device
    if dev not in _STREAMS:
        _STREAMS[dev] = torch.cuda.Stream(device=dev)
    return _STREAMS[dev]


def _comm_streams():
    """Raw handles of the communicator streams forked into a capture."""
    try:
        from ..distributed import _comm_stream_handles

        return _comm_stream_handles()
    except Exception:
        return []


class CapturedStep:
    def __init__(self, step_fn: Callable, static_inputs: Sequence[torch.Tensor], warmup: int = 3,
                 pool=None, stream: torch.cuda.Stream = None):
        self.step_fn = step_fn
        self.static_inputs = list(static_inputs)
        self.warmup = warmup
        self.pool = pool
        self.stream = stream or capture_stream()
        self.graph = None
        self.static_out = None
        self._capture()

    def _capture(self, warmup=None):
        s = self.stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup if warmup is None else warmup):
                self.step_fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(s)
        from ..parallel.ddp import finish_buffer_syncs

        with torch.cuda.stream(s):
            finish_buffer_syncs()  # the warmup's last forward may have left one in flight
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # thread_local: the communicator watchdog thread polls events while we
        # capture; in the default global mode that would invalidate the capture
        try:
            from ..ops.dropout import batched_offsets

            with torch.cuda.graph(g, pool=self.pool, stream=s, capture_error_mode="thread_local"):
                with batched_offsets():  # one dropout-counter advance per replay, not two nodes per call
                    self.static_out = self.step_fn(*self.static_inputs)
        except Exception:
            from .._ext import C as _C

            _C.abort_capture(s.cuda_stream)
            for extra in _comm_streams():
                _C.abort_capture(extra)
            raise
        self.graph = g

    def recapture(self, warmup: int = 0):
        """Capture again (e.g. after an LR change: the fused optimizers take
        hyper-parameters as kernel arguments). No warmup by default: capture
        itself executes nothing, so parameters are not advanced. The old graph
        stays alive until the new one is captured: a shared ``pool`` must be
        held by at least one graph when a capture begins into it (the caching
        allocator asserts on a pool whose last graph was destroyed)."""
        old = self.graph
        self._capture(warmup)
        del old

    def __call__(self, *inputs: torch.Tensor):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out
