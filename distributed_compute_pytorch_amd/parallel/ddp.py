"""DistributedDataParallel on the native Reducer.

Parity: ``torch.nn.parallel.DistributedDataParallel`` as constructed at
main.py:122 (``DistributedDataParallel(model, device_ids=[rank])``) —
SURVEY §2b F5, §3.2, §3.3. Same constructor arguments and semantics:

* construction: verify parameters across ranks (N6), broadcast parameters and
  buffers from rank 0 coalesced (F8, C2), plan buckets (F7) and build the C++
  Reducer (F6) that hooks every parameter's gradient accumulator;
* forward: broadcast buffers from rank 0 when ``broadcast_buffers`` and the
  previous forward was a synced training forward (C3), run the module, arm the
  Reducer for backward. With ``overlap_buffer_sync`` (default) that broadcast
  is started at the END of the synced forward, runs on the comm stream under
  the backward, and the next forward only unpacks it: the same values, no
  per-forward collective latency on the compute stream;
* backward: bucket all-reduces (average over the world) fire in bucket order
  while backward continues, finalize writes averaged gradients back;
* ``no_sync()``, ``register_comm_hook``, ``find_unused_parameters``,
  ``gradient_as_bucket_view``, and ``state_dict()`` keys with the ``module.``
  prefix (inherited from nn.Module).

MI355X specifics: the buckets are reduced by RCCL over xGMI on a dedicated
comm stream (no host sync in the step); pack/unpack are single HIP launches per
bucket; ``comm_dtype=torch.bfloat16`` halves the wire bytes (cast fused into
the pack launch).
"""
from __future__ import annotations

import contextlib
import warnings
from typing import Any, Callable, List, Optional

import torch
from torch import nn

from .._ext import C as _C
from .. import distributed as dist
from ..utils.trace import trace_range
from .comm_utils import CoalescedBroadcaster, broadcast_coalesced, verify_params_across_processes

# Constructor defaults = torch's (reducer.hpp:30-31): 25 MiB cap, 1 MiB first
# bucket, no tail split — a drop-in DDP plans the same buckets (and hands comm
# hooks the same bucket indices) as torch.nn.parallel.DistributedDataParallel.
DEFAULT_BUCKET_CAP_MB = 25.0
DEFAULT_FIRST_BUCKET_MB = 1.0
DEFAULT_TAIL_BUCKET_MB = 0.0

# xGMI-tuned plan for 8x MI355X, opted into by bench.py / train.py /
# workloads via ``DistributedDataParallel(..., **XGMI_BUCKETS)``. Chosen from
# the one-GPU contention-emulated sweep of an 8-rank ring all-reduce at
# 300 GB/s bus bandwidth (NOTES §25, profiles/r4_bucket_sweep_emulated.jsonl;
# cap 4-100 MiB x first bucket 0.25 / 1 / 4 MiB x tail 0 / 2 / 8 MiB, ResNet-50,
# BERT-base, GPT-2):
# * cap 16 MiB: the lowest or equal-lowest step time of all three models and
#   exposed (un-overlapped) comm ResNet-50 0.05 ms, BERT 1.27, GPT-2 2.31 ms
#   vs 0.055 / 1.58 / 2.89 at 50 MiB — smaller buckets start reducing earlier
#   and leave less queued behind the ready-last ones; below 16 MiB the pack
#   launches and per-collective latency cost ResNet-50 0.06-0.09 ms exposed;
# * first bucket 1 MiB: 0.25 / 1 / 4 MiB measured the same (within 0.01 ms);
# * tail 2 MiB: the ready-last parameters in a latency-bound bucket of their
#   own — without it ResNet-50 exposes 0.11 (cap 25) / 0.38 ms (cap 50).
XGMI_BUCKETS = {"bucket_cap_mb": 16.0, "first_bucket_mb": 1.0, "tail_bucket_mb": 2.0}


# overlap-mode DDP instances (optim/fused.py syncs their deferred buckets
# chunk by chunk inside the optimizer step)
import weakref as _weakref

_OVERLAP = _weakref.WeakSet()


class _PendingGrad(torch.Tensor):
    """``.grad`` of a parameter whose bucket reduction is still in flight
    (``overlap_optimizer=True``): the bucket view itself (same storage), but
    any torch operation on it — a stock ``torch.optim`` step, ``torch.nn.
    utils.clip_grad_norm_``, a GradScaler, ``zero_grad(set_to_none=False)``,
    user code — first orders the caller behind the reduction (device-side
    event wait on RCCL, a host wait on the host backend) and rebinds the
    parameters' ``.grad`` to the plain views; the op then runs on the reduced
    values. Only this package's fused optimizers read the pending views
    without that sync: they sync bucket by bucket, in launch order, right
    before updating each bucket's parameters (the overlap)."""

    @staticmethod
    def wrap(view: torch.Tensor, ddp, k: int) -> "_PendingGrad":
        t = view.as_subclass(_PendingGrad)
        t._dcp_src = (_weakref.ref(ddp), k)
        t._dcp_plain = view  # the fused optimizers read this after their own per-bucket sync
        return t

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        seen = set()

        def visit(a):
            if isinstance(a, _PendingGrad):
                src = a.__dict__.get("_dcp_src")
                if src is not None and (id(src[0]), src[1]) not in seen:
                    seen.add((id(src[0]), src[1]))
                    d = src[0]()
                    if d is not None:
                        d._sync_bucket(src[1])
            elif isinstance(a, (list, tuple)):
                for x in a:
                    visit(x)
            elif isinstance(a, dict):
                for x in a.values():
                    visit(x)

        visit(args)
        visit(kwargs)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)


_DTYPE_IDS = {torch.float32: 0, torch.float64: 1, torch.float16: 2, torch.bfloat16: 3, torch.int64: 4,
              torch.int32: 5, torch.uint8: 6, torch.int8: 7, torch.bool: 8, torch.complex64: 9}


class GradBucket:
    """Argument of a comm hook: the flat bucket buffer (torch-like accessors).
    ``index()`` is the bucket's position in the current iteration's launch
    order (0 = first reduced), as in torch's ``GradBucket.index()``."""

    def __init__(self, buffer: torch.Tensor, index: int, params: Optional[List[torch.Tensor]] = None,
                 num_buckets: int = 0):
        self._buffer = buffer
        self._index = index
        self._params = params or []
        self._num_buckets = num_buckets

    def buffer(self) -> torch.Tensor:
        return self._buffer

    def index(self) -> int:
        return self._index

    def is_last(self) -> bool:
        return self._index == self._num_buckets - 1

    def parameters(self) -> List[torch.Tensor]:
        return list(self._params)

    def set_buffer(self, tensor: torch.Tensor) -> None:
        self._buffer.copy_(tensor)


_BUFFER_SYNCS = _weakref.WeakSet()  # DDPs that may hold an overlapped buffer broadcast in flight


def finish_buffer_syncs() -> None:
    """Complete every overlapped buffer broadcast still in flight (before a
    HIP-graph capture: a captured forward must not wait on work enqueued
    outside the capture)."""
    for d in list(_BUFFER_SYNCS):
        if d._buffer_bcast is not None and d._buffer_bcast.pending:
            d._buffer_bcast.finish()


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids: Optional[List[Any]] = None, output_device=None, dim: int = 0,
                 broadcast_buffers: bool = True, process_group=None, bucket_cap_mb: Optional[float] = None,
                 find_unused_parameters: bool = False, check_reduction: bool = False,
                 gradient_as_bucket_view: bool = False, static_graph: bool = False,
                 first_bucket_mb: Optional[float] = None, comm_dtype: Optional[torch.dtype] = None,
                 rebuild_buckets: bool = True, init_sync: bool = True, tail_bucket_mb: Optional[float] = None,
                 register_buckets: bool = False, overlap_optimizer: bool = False, defer_accum_wgrad: bool = False,
                 overlap_buffer_sync: bool = True, bucket_slice_mb: Optional[float] = None):
        super().__init__()
        self.module = module
        self.process_group = process_group if process_group is not None else dist.get_default_group()
        if check_reduction:
            # torch deprecated and ignores it; so do we, but not silently
            warnings.warn("DistributedDataParallel: check_reduction is deprecated and has no effect (as in torch)",
                          FutureWarning, stacklevel=2)
        if not isinstance(dim, int) or isinstance(dim, bool):
            raise TypeError(f"DistributedDataParallel: dim must be an int, got {dim!r}")
        self.device_ids = device_ids
        # the input scatter dimension of torch's multi-device mode; a module
        # lives on ONE device here (one process per GPU), where torch does not
        # scatter either, so dim has no effect beyond this validation
        self.dim = dim
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.gradient_as_bucket_view = gradient_as_bucket_view
        self.static_graph = static_graph
        self.require_backward_grad_sync = True
        self.require_forward_param_sync = True
        self.bucket_bytes_cap = int((bucket_cap_mb if bucket_cap_mb is not None else DEFAULT_BUCKET_CAP_MB) * 2**20)
        self.first_bucket_bytes = int(
            (first_bucket_mb if first_bucket_mb is not None else DEFAULT_FIRST_BUCKET_MB) * 2**20)
        self.tail_bucket_bytes = int((tail_bucket_mb if tail_bucket_mb is not None else DEFAULT_TAIL_BUCKET_MB) * 2**20)

        # unique trainable parameters in registration order
        seen = set()
        params = []
        for p in module.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        if not params:
            raise RuntimeError("DistributedDataParallel: module has no parameter that requires gradient")
        devs = {p.device for p in params}
        if len(devs) != 1:
            raise ValueError(f"DistributedDataParallel expects the module on one device, found {devs}")
        self.device = next(iter(devs))
        if device_ids is not None:
            if len(device_ids) != 1:
                raise ValueError("DistributedDataParallel: one process per device — device_ids must hold exactly "
                                 f"one device, got {device_ids!r}")
            if self.device.type != "cuda" or torch.device("cuda", _dev_index(device_ids[0])) != self.device:
                raise ValueError(f"DistributedDataParallel: device_ids={device_ids!r} but the module's parameters "
                                 f"are on {self.device}")
        if output_device is not None:
            od = torch.device("cuda", output_device) if isinstance(output_device, int) else torch.device(output_device)
            if od.type == "cuda" and od.index is None:
                od = torch.device("cuda", torch.cuda.current_device())
            if od != self.device:
                raise ValueError(f"DistributedDataParallel: output_device={output_device!r} differs from the module's "
                                 f"device {self.device}; single-device modules return outputs where they are")
        self.output_device = output_device
        self._params = params
        self._buffers_list = [b for b in module.buffers()]

        pg = self.process_group
        verify_params_across_processes(pg, params)
        if init_sync:
            broadcast_coalesced(pg, [p.detach() for p in params] + [b for b in self._buffers_list], 0)
        self._buffer_bcast = CoalescedBroadcaster(self._buffers_list) if self._buffers_list else None
        # overlap_buffer_sync: the buffer broadcast a synchronising forward
        # would make the NEXT forward wait for is started right after this one
        # (rank 0's buffers as this forward left them) and runs on the
        # communicator's stream under the backward; the next forward only
        # unpacks it. Those are the values torch's start-of-forward broadcast
        # would deliver, unless rank 0's buffers change between the forwards
        # outside a forward (then call sync_buffers() first). Off: the
        # broadcast runs at the start of the forward, as torch's does.
        self.overlap_buffer_sync = bool(overlap_buffer_sync)
        if self._buffer_bcast is not None:
            # buffers replaced by load_state_dict (e.g. on resume) must not be
            # overwritten by the broadcast of rank 0's pre-load values still in
            # flight: its result is dropped (the collective itself still
            # completes on every rank, so ranks that did not load stay in step)
            me_ = _weakref.ref(self)

            def _loaded(_module, _keys):
                d = me_()
                if d is not None and d._buffer_bcast.pending:
                    d._buffer_bcast.discard()

            module.register_load_state_dict_post_hook(_loaded)

        # Initial plan: registration order, [first, cap] limits, then reversed so
        # the bucket holding the last-defined parameters (ready first) is bucket 0.
        sizes = [p.numel() * p.element_size() for p in params]
        keys = [self._key(p) for p in params]
        plan = _C.compute_bucket_assignment(sizes, keys, [self.first_bucket_bytes, self.bucket_bytes_cap], [])
        # expected-ready order: buckets AND their members reversed (gradients
        # arrive roughly in reverse registration order)
        plan = [list(reversed(b)) for b in reversed(plan)]
        plan = _C.split_tail_bucket(plan, sizes, self.tail_bucket_bytes)
        opts = _C.ReducerOptions()
        opts.gradient_as_bucket_view = gradient_as_bucket_view
        # static_graph (torch's flag): the used-parameter set of the first
        # synchronised backward is reused every iteration — unused parameters
        # are handled without find_unused_parameters' per-step traversal and
        # used-map collective (reducer.cpp "static_graph"). The graph must not
        # change between iterations (as in torch).
        opts.find_unused_parameters = find_unused_parameters or static_graph
        opts.static_graph = bool(static_graph)
        opts.rebuild_buckets = rebuild_buckets
        opts.first_bucket_bytes = self.first_bucket_bytes
        opts.bucket_bytes_cap = self.bucket_bytes_cap
        opts.tail_bucket_bytes = self.tail_bucket_bytes
        if comm_dtype is not None:
            opts.comm_dtype = comm_dtype
        # register_buckets: the bucket buffers are registered with RCCL
        # (ncclCommRegister) once per bucket plan — zero-copy user-buffer paths
        # where RCCL has them; a no-op on one rank and on gloo
        opts.register_buckets = bool(register_buckets)
        # overlap_optimizer: the backward leaves the last bucket reductions in
        # flight; this package's fused optimizers (optim/fused.py) order the
        # compute stream behind each bucket right before updating its
        # parameters, so the update of the early buckets overlaps the
        # reduction of the last ones (the ready-last embeddings of BERT /
        # GPT-2 are single 90-150 MB buckets). Needs gradient_as_bucket_view
        # (the gradients ARE the bucket buffers); anything else reading .grad
        # between backward and step must call wait_gradients() first.
        self.overlap_optimizer = bool(overlap_optimizer) and gradient_as_bucket_view and not find_unused_parameters
        # (static_graph: deferred from the second iteration on, when every
        # parameter was used somewhere in the first)
        opts.defer_grad_wait = self.overlap_optimizer
        # bucket_slice_mb (overlap_optimizer): a bucket over 1.5x this size is
        # reduced as several collectives over slices of its buffer, and the
        # fused Adam updates each slice's parameter ranges as soon as that
        # slice lands — the single-parameter tied-embedding buckets (GPT-2
        # 147 MB, BERT 89 MB) are ready last, so otherwise their whole
        # reduction is exposed before their update can start. Default: the
        # bucket cap, at least 4 MB; 0 = one collective per bucket.
        if bucket_slice_mb is None:
            bucket_slice_mb = max(self.bucket_bytes_cap / 2**20, 4.0) if self.overlap_optimizer else 0.0
        if bucket_slice_mb < 0:
            raise ValueError(f"DistributedDataParallel: bucket_slice_mb must be >= 0, got {bucket_slice_mb}")
        self.bucket_slice_bytes = int(bucket_slice_mb * 2**20) if self.overlap_optimizer else 0
        opts.slice_bytes = self.bucket_slice_bytes
        # defer_accum_wgrad: under no_sync the Linear weight gradients of the
        # micro-steps are not computed one by one; the synchronising micro-step
        # computes each over all micro-steps' rows in one launch (ops/linear.py
        # "micro-step weight-gradient deferral"). p.grad of those weights lacks
        # the no_sync contributions until that backward or an optimizer step.
        self.defer_accum_wgrad = bool(defer_accum_wgrad)
        if self.defer_accum_wgrad and self.process_group.size() > 1:
            from ..ops import linear as _lin

            _lin._MULTI_RANK_DEFER[0] += 1
        self._comm = pg.comm_for(params[0])
        self.reducer = _C.Reducer(params, plan, self._comm, opts)
        self._comm_hook = None
        if self.overlap_optimizer:
            _OVERLAP.add(self)
            me = _weakref.ref(self)
            cache = {}  # bucket -> (view data pointers, wrappers): the views persist across iterations

            def _wrap(k, views):
                d = me()
                if d is None:
                    return list(views)
                ptrs = tuple(v.data_ptr() for v in views)
                hit = cache.get(k)
                if hit is None or hit[0] != ptrs:
                    hit = cache[k] = (ptrs, [_PendingGrad.wrap(v, d, k) for v in views])
                return hit[1]

            self.reducer.set_deferred_grad_hook(_wrap)
            _install_step_sync_hook()

    @staticmethod
    def _key(p):
        dev = p.device
        # deterministic across processes (ranks must plan identically)
        return _DTYPE_IDS.get(p.dtype, 255) << 32 | (0 if dev.type == "cpu" else 1) << 16 | ((dev.index or 0) + 1)

    # ------------------------------------------------------------------
    def forward(self, *inputs, **kwargs):
        with trace_range("DistributedDataParallel.forward"):
            return self._forward(*inputs, **kwargs)

    def _forward(self, *inputs, **kwargs):
        grad = torch.is_grad_enabled()
        bufs = self.broadcast_buffers and self._buffer_bcast is not None and self.process_group.size() > 1
        if bufs:
            if self._buffer_bcast.pending:  # started after the previous (synchronising) forward
                self._buffer_bcast.finish()
            elif self.require_forward_param_sync:
                self._buffer_bcast(self.process_group, 0)
        if self.device_ids is not None:
            # torch moves the inputs to device_ids[0] (main.py passes them there already)
            inputs, kwargs = _to_device(inputs, self.device), _to_device(kwargs, self.device)
        out = self.module(*inputs, **kwargs)
        if grad and self.require_backward_grad_sync:
            if self.defer_accum_wgrad:
                # pending no_sync segments this forward's Linears will not
                # consume go into .grad now, inside the bucket reduction
                from ..ops.linear import flush_unclaimed

                flushed = flush_unclaimed(self._params)
                if flushed and (self.find_unused_parameters or self.static_graph):
                    # used in this accumulation round, even if not in this backward
                    pos = self.__dict__.setdefault("_pos", {id(p): i for i, p in enumerate(self._params)})
                    self.reducer.note_used([pos[id(p)] for p in flushed if id(p) in pos])
            self.require_forward_param_sync = True
            if bufs and self.overlap_buffer_sync and not (self.device.type == "cuda"
                                                           and torch.cuda.is_current_stream_capturing()):
                self._buffer_bcast.start(self.process_group, 0)
                _BUFFER_SYNCS.add(self)
            traverse = self.find_unused_parameters or (self.static_graph and not self.reducer.static_frozen)
            outs = _tensors_in(out) if traverse else []
            self.reducer.prepare_for_backward(outs, True)
        else:
            self.require_forward_param_sync = False
            self.reducer.prepare_for_backward([], False)
        return out

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (no all-reduce) inside the context."""
        from ..ops.linear import accumulate_grads_in_place, defer_weight_grads

        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            with accumulate_grads_in_place(), (defer_weight_grads() if self.defer_accum_wgrad
                                               else contextlib.nullcontext()):
                yield
        finally:
            self.require_backward_grad_sync = old

    def register_comm_hook(self, state: object, hook: Callable):
        """``hook(state, bucket: GradBucket) -> Work | None``; the hook must leave
        the reduced (averaged) gradient in ``bucket.buffer()`` once its Work
        completes. See :mod:`.comm_hooks` for the built-ins."""
        if self._comm_hook is not None:
            raise RuntimeError("register_comm_hook can only be called once")
        self._comm_hook = hook
        reducer, params = self.reducer, self._params

        def _call(buf, idx):
            plan = reducer.bucket_indices()
            ps = [params[i] for i in plan[idx]] if idx < len(plan) else []
            return hook(state, GradBucket(buf, idx, ps, len(plan)))

        # a compression hook declares its wire precision (``hook.wire_dtype``):
        # the debug stream-ordering check then tolerates that rounding
        self.reducer.set_comm_hook(_call, getattr(hook, "wire_dtype", None))

    def sync_buffers(self) -> None:
        """Broadcast the module's buffers from rank 0 now (after completing an
        overlapped broadcast still in flight). Collective: every rank calls it."""
        if self._buffer_bcast is None or self.process_group.size() == 1:
            return
        if self._buffer_bcast.pending:
            self._buffer_bcast.finish()
        self._buffer_bcast(self.process_group, 0)

    def set_comm_timing(self, on: bool) -> None:
        """Device-time instrumentation of the bucket collectives (what
        ``DCP_COMM_TIMING=1`` turns on at construction) from the next
        backward on: ``ddp_logging_data()``'s bucket_comm_ms /
        bucket_ready_dev_ms / exposed_comm_ms."""
        self._comm.set_timing(bool(on))
        self.reducer.set_timing(bool(on))

    def wait_gradients(self) -> None:
        """overlap_optimizer: order the current stream behind every bucket
        reduction still in flight and hand out the plain gradient views (any
        torch op on a pending ``.grad`` does this by itself)."""
        self.reducer.sync_all()
        self._unwrap(range(len(self.reducer.bucket_indices())))

    def _sync_bucket(self, k: int) -> None:
        """overlap_optimizer: order the current stream behind bucket k's
        reduction and rebind its parameters' ``.grad`` to the plain views."""
        self.reducer.sync_bucket(k)
        self._unwrap((k,))

    def _unwrap(self, ks) -> None:
        plan = self.reducer.bucket_indices()
        with torch._C.DisableTorchFunctionSubclass():
            for k in ks:
                if k >= len(plan):
                    continue
                for i in plan[k]:
                    p = self._params[i]
                    g = p.grad
                    if isinstance(g, _PendingGrad):
                        p.grad = g.as_subclass(torch.Tensor)

    # ------------------------------------------------------------------
    def bucket_sizes(self) -> List[int]:
        return list(self.reducer.bucket_sizes_bytes())

    def ddp_logging_data(self) -> dict:
        st = self.reducer.bucket_stats()
        return {
            "world_size": self.process_group.size(),
            "backend": self._comm.backend,
            "bucket_cap_bytes": self.bucket_bytes_cap,
            "first_bucket_bytes": self.first_bucket_bytes,
            "tail_bucket_bytes": self.tail_bucket_bytes,
            "bucket_sizes": [s.bytes for s in st],
            "bucket_ready_ms": [s.ready_ms for s in st],  # host enqueue time (1 ms resolution)
            # DCP_COMM_TIMING=1: device time from the backward's first gradient
            # hook to each bucket's packed gradients (-1 without timing)
            "bucket_ready_dev_ms": [s.ready_dev_ms for s in st],
            "bucket_comm_ms": [s.comm_ms for s in st],
            "num_buckets": len(st),
            "bucket_indices": self.reducer.bucket_indices(),
            "iterations": self.reducer.num_iterations,
            "rebuilds": self.reducer.num_rebuilds,
            "comm_ops": self._comm.ops_issued,
            "comm_bytes": self._comm.bytes_issued,
            # DCP_COMM_TIMING=1: reduction time not hidden behind backward
            "exposed_comm_ms": self.reducer.exposed_comm_ms(),
        }


_STEP_HOOK = [False]


def _install_step_sync_hook():
    """Before any optimizer step that is not one of this package's fused
    optimizers (they sync bucket by bucket themselves): sync every
    overlap-mode DDP. (A torch op on a pending .grad syncs anyway; this also
    covers optimizers that hand the gradients to native code directly.)"""
    if _STEP_HOOK[0]:
        return
    from torch.optim.optimizer import register_optimizer_step_pre_hook

    def hook(opt, args, kwargs):
        from ..optim import fused

        if isinstance(opt, (fused.SGD, fused.Adam, fused.Adadelta)):
            return
        for d in list(_OVERLAP):
            d.wait_gradients()

    register_optimizer_step_pre_hook(hook)
    _STEP_HOOK[0] = True


def _dev_index(d) -> int:
    if isinstance(d, int):
        return d
    d = torch.device(d)
    return d.index if d.index is not None else torch.cuda.current_device()


def _to_device(obj, device):
    """``obj`` with every tensor in it (through tuples, lists and dicts) on ``device``."""
    if isinstance(obj, torch.Tensor):
        return obj if obj.device == device else obj.to(device, non_blocking=True)
    if isinstance(obj, tuple) and hasattr(obj, "_fields"):  # namedtuple
        return type(obj)(*(_to_device(o, device) for o in obj))
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_device(o, device) for o in obj)
    if isinstance(obj, dict):
        return type(obj)((k, _to_device(v, device)) for k, v in obj.items())
    return obj


def _tensors_in(obj):
    out = []
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            out.extend(_tensors_in(o))
    elif isinstance(obj, dict):
        for o in obj.values():
            out.extend(_tensors_in(o))
    return out
