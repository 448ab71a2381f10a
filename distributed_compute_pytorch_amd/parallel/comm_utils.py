"""Coalesced broadcast / parameter verification helpers.

Parity: torch's ``_broadcast_coalesced`` (comm.cpp) and
``_verify_param_shape_across_processes`` that DDP runs at construction and,
for buffers, every training forward.
Flatten/unflatten is one multi-tensor HIP launch per dtype group
(``_C.mt_copy``), the broadcast one RCCL call per group.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Sequence

import torch

from .._ext import C as _C

_MT_DTYPES = (torch.float32, torch.bfloat16, torch.float16)


def is_dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (any dim permutation), like ATen's check."""
    if t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)):
        return True
    expected = 1
    for size, stride in sorted(zip(t.shape, t.stride()), key=lambda a: a[1]):
        if size == 1:
            continue
        if stride != expected:
            return False
        expected *= size
    return True


def _group_by_dtype(tensors: Sequence[torch.Tensor]):
    groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
    for i, t in enumerate(tensors):
        groups.setdefault((t.dtype, t.device), []).append(i)
    return groups


def _flat_views(flat: torch.Tensor, tensors: Sequence[torch.Tensor]):
    views, off = [], 0
    for t in tensors:
        n = t.numel()
        views.append(flat.as_strided(t.shape, t.stride(), off) if is_dense(t)
                     else flat[off:off + n].view(t.shape))
        off += n
    return views


_WORD_VIEW = {torch.int64: torch.float32, torch.float64: torch.float32, torch.int32: torch.float32,
              torch.int16: torch.bfloat16}


def _as_words(ts: Sequence[torch.Tensor]):
    """Bit-preserving float32/bf16 views of 2/4/8-byte tensors (for the raw
    multi-tensor copy): one launch moves every buffer regardless of dtype."""
    out = []
    for t in ts:
        wd = _WORD_VIEW.get(t.dtype, t.dtype)
        if wd is t.dtype:
            out.append(t)
        elif t.is_contiguous():
            out.append(t.reshape(-1).view(wd))
        else:
            return None
    return out


def _copy_list(src: Sequence[torch.Tensor], dst: Sequence[torch.Tensor]):
    if src and src[0].is_cuda and all(is_dense(t) for t in list(src) + list(dst)) \
            and all(s.dtype == d.dtype for s, d in zip(src, dst)):
        ws, wd = _as_words(src), _as_words(dst)
        if ws is not None and wd is not None and all(t.dtype in _MT_DTYPES for t in ws):
            _C.mt_copy(ws, wd, 1.0)  # same dtype, scale 1 -> bit-exact raw copy kernel
            return
    if src and not src[0].is_cuda and all(s.dtype == d.dtype for s, d in zip(src, dst)) and \
            all(t.dtype in _MT_DTYPES for t in src) and all(is_dense(t) for t in list(src) + list(dst)):
        _C.mt_copy(list(src), list(dst), 1.0)
        return
    for s, d in zip(src, dst):
        d.copy_(s)


def pack(tensors: Sequence[torch.Tensor], flat: torch.Tensor):
    _copy_list(list(tensors), _flat_views(flat, tensors))


def unpack(flat: torch.Tensor, tensors: Sequence[torch.Tensor]):
    _copy_list(_flat_views(flat, tensors), list(tensors))


def _word_key(t: torch.Tensor):
    """The group a tensor is broadcast in: contiguous tensors of 4- / 8-byte
    dtypes travel as float32 words (a broadcast moves bits, so BatchNorm's
    fp32 running stats and int64 ``num_batches_tracked`` share ONE collective),
    everything else by its own dtype."""
    if t.is_contiguous() and t.element_size() in (4, 8) and t.dtype in (torch.float32, torch.int64, torch.float64,
                                                                          torch.int32):
        return torch.float32, t.device
    return t.dtype, t.device


class CoalescedBroadcaster:
    """Broadcast a fixed list of tensors from ``src`` with one collective per
    word group (``_word_key``: ResNet's BatchNorm buffers are ONE broadcast per
    forward); flat buffers are allocated once and reused (the per-forward
    buffer broadcast is latency-bound)."""

    def __init__(self, tensors: Sequence[torch.Tensor], cap_bytes: int = 250 << 20):
        self.tensors = list(tensors)
        self.cap = cap_bytes
        self.plan = []  # list of (indices, flat)
        self._pending = None  # (works, unpack?) between start() and finish()
        groups: "OrderedDict[tuple, List[int]]" = OrderedDict()
        for i, t in enumerate(self.tensors):
            groups.setdefault(_word_key(t), []).append(i)
        for (dtype, device), idx in groups.items():
            chunk, size = [], 0
            for i in idx:
                nb = self.tensors[i].numel() * self.tensors[i].element_size()
                if chunk and size + nb > self.cap:
                    self.plan.append(self._mk(chunk, dtype, device))
                    chunk, size = [], 0
                chunk.append(i)
                size += nb
            if chunk:
                self.plan.append(self._mk(chunk, dtype, device))

    def _mk(self, idx, dtype, device):
        n = sum(self.tensors[i].numel() * self.tensors[i].element_size() for i in idx) // torch.empty(
            0, dtype=dtype).element_size()
        return idx, torch.empty(n, dtype=dtype, device=device)

    def _views(self, idx, flat):
        """The group's tensors as views of ``flat``'s dtype (bit-preserving)."""
        out = []
        for i in idx:
            t = self.tensors[i]
            out.append(t if t.dtype == flat.dtype else t.reshape(-1).view(flat.dtype))
        return out

    @torch.no_grad()
    def start(self, pg, src: int = 0):
        """Pack (on ``src``) and enqueue the broadcasts; :meth:`finish` waits
        and unpacks. Between the two the collectives run on the communicator's
        stream while the caller's stream goes on (the flat buffers are owned
        here, so nothing the caller does touches them)."""
        if self._pending is not None:
            raise RuntimeError("CoalescedBroadcaster: start() while a broadcast is pending")
        works = []
        for idx, flat in self.plan:
            if pg.rank() == src:
                pack(self._views(idx, flat), flat)
            works.append((pg.comm_for(flat).broadcast(flat, src), idx, flat))
        self._pending = (works, pg.rank() != src)

    @property
    def pending(self) -> bool:
        return self._pending is not None

    @torch.no_grad()
    def finish(self):
        works, recv = self._pending
        self._pending = None
        for w, idx, flat in works:
            w.wait()
            if recv:
                unpack(flat, self._views(idx, flat))

    def discard(self):
        """Keep the pending broadcast (every rank still completes the same
        collectives in :meth:`finish`), but do not unpack its result: no tensor
        is overwritten with the values it carries."""
        works, _ = self._pending
        self._pending = (works, False)

    def __call__(self, pg, src: int = 0):
        self.start(pg, src)
        self.finish()


def broadcast_coalesced(pg, tensors: Sequence[torch.Tensor], src: int = 0, cap_bytes: int = 250 << 20):
    if pg.size() == 1 or not tensors:
        return
    CoalescedBroadcaster(tensors, cap_bytes)(pg, src)


def verify_params_across_processes(pg, params: Sequence[torch.Tensor]):
    """All ranks must hold the same parameter list (count, shapes, dtypes):
    otherwise the bucket collectives would mismatch and hang."""
    if pg.size() == 1:
        return
    desc = ";".join(f"{tuple(p.shape)}:{p.dtype}:{tuple(p.stride())}" for p in params)
    digest = hashlib.sha1(desc.encode()).hexdigest()
    key = f"{pg.prefix}/ddp/verify/{_verify_seq.setdefault(pg.prefix, 0)}"
    _verify_seq[pg.prefix] += 1
    pg.store.set(f"{key}/{pg.rank()}", f"{len(params)}|{digest}".encode())
    mine = f"{len(params)}|{digest}"
    for r in range(pg.size()):
        other = pg.store.get(f"{key}/{r}").decode()
        if other != mine:
            raise RuntimeError(
                f"DDP: rank {pg.rank()} has parameters [{mine}] but rank {r} has [{other}]; every rank must "
                "construct the same model")


_verify_seq: Dict[str, int] = {}
