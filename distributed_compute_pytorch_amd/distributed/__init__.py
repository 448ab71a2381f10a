"""torch.distributed-compatible collective API on the native runtime.

Parity: the reference calls
``dist.init_process_group("gloo", rank=rank, world_size=world_size)``
(main.py:50), ``dist.all_reduce(t, op=dist.ReduceOp.SUM)`` (main.py:65,
main.py:90-91) and ``dist.destroy_process_group()`` (main.py:53). The same
calls work here:

* rendezvous: env:// (MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE) or
  tcp://host:port, over the C++ ``TCPStore`` (rank 0 hosts the server);
* backends: ``"rccl"`` (alias ``"nccl"``) — device tensors over RCCL/xGMI on a
  dedicated comm stream; ``"host"`` (alias ``"gloo"``) — the C++ TCP ring
  communicator for CPU tensors (device tensors are staged through host memory,
  the reference-literal mode); ``"auto"`` — RCCL for device tensors when a GPU
  is present, host for CPU tensors. One communicator per device type, created
  lazily.
"""
from __future__ import annotations

import datetime as _dt
import os
import pickle
from typing import List, Optional

import torch

from .._ext import C as _C

__all__ = [
    "ReduceOp",
    "ProcessGroup",
    "GroupMember",
    "init_process_group",
    "destroy_process_group",
    "is_initialized",
    "is_available",
    "get_rank",
    "get_world_size",
    "get_backend",
    "new_group",
    "all_reduce",
    "broadcast",
    "all_gather",
    "all_gather_into_tensor",
    "reduce_scatter",
    "reduce_scatter_tensor",
    "all_to_all_single",
    "send",
    "recv",
    "isend",
    "irecv",
    "barrier",
    "broadcast_object_list",
    "all_gather_object",
    "get_default_group",
    "Work",
]

Work = _C.Work
_DEFAULT_TIMEOUT = _dt.timedelta(minutes=30)


class ReduceOp:
    SUM = _C.ReduceOp.SUM
    AVG = _C.ReduceOp.AVG
    PRODUCT = _C.ReduceOp.PRODUCT
    MIN = _C.ReduceOp.MIN
    MAX = _C.ReduceOp.MAX


def _to_op(op):
    if isinstance(op, _C.ReduceOp):
        return op
    # accept torch.distributed.ReduceOp values / names
    name = getattr(op, "name", None) or str(op).split(".")[-1]
    name = name.upper()
    table = {"SUM": ReduceOp.SUM, "AVG": ReduceOp.AVG, "PRODUCT": ReduceOp.PRODUCT, "MIN": ReduceOp.MIN,
             "MAX": ReduceOp.MAX}
    if name not in table:
        raise ValueError(f"unsupported reduce op {op!r}")
    return table[name]


_BACKEND_ALIASES = {"nccl": "rccl", "rccl": "rccl", "gloo": "host", "host": "host", "auto": "auto", "cpu": "host"}


class ProcessGroup:
    """A set of ranks sharing communicators (one per device type)."""

    def __init__(self, store, prefix: str, rank: int, size: int, backend: str, timeout_ms: int,
                 global_ranks: List[int], device_id: Optional[int] = None):
        self.store = store
        self.prefix = prefix
        self._rank = rank
        self._size = size
        self.backend = backend
        self.timeout_ms = timeout_ms
        self.global_ranks = list(global_ranks)
        self.device_id = device_id
        self._host = None
        self._rccl = None
        self._debug_fp = os.environ.get("DCP_DEBUG_COLLECTIVES") == "1"
        self._obj_seq = 0  # object-collective calls on this group (store key sequence)

    def rank(self) -> int:
        return self._rank

    def size(self) -> int:
        return self._size

    # -- communicators ---------------------------------------------------
    def host_comm(self):
        if self._host is None:
            self._host = _C.make_host_communicator(self.store, self.prefix, self._rank, self._size,
                                                   self.timeout_ms)
            self._host.set_debug_fingerprint(self._debug_fp)
        return self._host

    def rccl_comm(self, device: Optional[int] = None):
        if self._rccl is None:
            dev = device if device is not None else self.device_id
            if dev is None:
                dev = torch.cuda.current_device()
            self._rccl = _C.make_rccl_communicator(self.store, self.prefix, self._rank, self._size, int(dev),
                                                   self.timeout_ms)
            self._rccl.set_debug_fingerprint(self._debug_fp)
            self.device_id = int(dev)
        return self._rccl

    def comm_for(self, t: torch.Tensor):
        if t.is_cuda and self.backend in ("rccl", "auto"):
            return self.rccl_comm(t.get_device())
        if not t.is_cuda and self.backend == "rccl":
            raise RuntimeError("backend 'rccl' handles device tensors only; use backend='auto' or 'host' for CPU")
        return self.host_comm()

    def abort(self):
        for c in (self._rccl, self._host):
            if c is not None:
                c.abort()

    def __repr__(self):
        return f"ProcessGroup(rank={self._rank}, size={self._size}, backend={self.backend!r}, prefix={self.prefix!r})"


class _NonMember:
    def __repr__(self):
        return "GroupMember.NON_GROUP_MEMBER"


class GroupMember:
    WORLD = None
    NON_GROUP_MEMBER = _NonMember()


_state = {"default": None, "groups": [], "group_count": 0}


def _comm_stream_handles() -> List[int]:
    """Raw HIP stream handles of every live RCCL communicator (graph-capture recovery)."""
    out = []
    for pg in [_state["default"], *_state["groups"]]:
        if pg is not None and pg._rccl is not None:
            out.append(int(pg._rccl.stream_handle))
    return out


def is_available() -> bool:
    return True


def is_initialized() -> bool:
    return _state["default"] is not None


def get_default_group() -> ProcessGroup:
    pg = _state["default"]
    if pg is None:
        raise RuntimeError("Default process group has not been initialized; call init_process_group first")
    return pg


def _group(group) -> ProcessGroup:
    if group is None or group is GroupMember.WORLD:
        return get_default_group()
    if group is GroupMember.NON_GROUP_MEMBER:
        raise RuntimeError("this rank is not a member of the group")
    return group


def _parse_init(init_method: str, rank: int, world_size: int):
    if init_method is None or init_method == "env://":
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        if rank < 0:
            rank = int(os.environ["RANK"])
        if world_size < 0:
            world_size = int(os.environ["WORLD_SIZE"])
        return addr, port, rank, world_size
    if init_method.startswith("tcp://"):
        hostport = init_method[len("tcp://"):].split("?")[0]
        host, port = hostport.rsplit(":", 1)
        if rank < 0 or world_size < 0:
            raise ValueError("tcp:// init needs explicit rank and world_size")
        return host, int(port), rank, world_size
    raise ValueError(f"unsupported init_method {init_method!r}")


def _bootstrap_from_agent_store(addr: str, port: int, rank: int, world_size: int, timeout_ms: int):
    """Under torchrun / torch.distributed.run the elastic agent already hosts a
    (torch) TCPStore on MASTER_ADDR:MASTER_PORT. Rank 0 starts our C++ store on
    an ephemeral port and publishes it through the agent's store; the other
    ranks read it and connect. (Same-protocol reuse is impossible: the agent
    store speaks torch's wire format.)"""
    import datetime

    import torch.distributed as tdist

    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    key = f"dcp/store_addr/{attempt}"
    agent = tdist.TCPStore(addr, port, world_size, False, timeout=datetime.timedelta(milliseconds=timeout_ms))
    if rank == 0:
        ours = _C.TCPStore(addr, 0, world_size, True, timeout_ms, False)
        agent.set(key, f"{ours.local_ip()}:{ours.port}")
    else:
        host, p = agent.get(key).decode().rsplit(":", 1)
        ours = _C.TCPStore(host, int(p), world_size, False, timeout_ms, False)
    ours.barrier("init")
    return ours


def init_process_group(backend: Optional[str] = None, init_method: Optional[str] = None,
                       timeout: Optional[_dt.timedelta] = None, world_size: int = -1, rank: int = -1,
                       store=None, group_name: str = "", pg_options=None, device_id=None) -> None:
    """Create the default process group (same signature as torch.distributed)."""
    if is_initialized():
        raise RuntimeError("trying to initialize the default process group twice")
    be = _BACKEND_ALIASES.get((backend or "auto").lower())
    if be is None:
        raise ValueError(f"unknown backend {backend!r}; use 'rccl'/'nccl', 'host'/'gloo' or 'auto'")
    timeout_ms = int((timeout or _DEFAULT_TIMEOUT).total_seconds() * 1000)
    if store is None:
        addr, port, rank, world_size = _parse_init(init_method, rank, world_size)
        if (init_method in (None, "env://") and
                os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() in ("true", "1")):
            store = _bootstrap_from_agent_store(addr, port, rank, world_size, timeout_ms)
        else:
            store = _C.TCPStore(addr, port, world_size, rank == 0, timeout_ms, True)
    else:
        if rank < 0 or world_size < 0:
            raise ValueError("explicit store needs rank and world_size")
    if isinstance(device_id, torch.device):
        device_id = device_id.index
    if device_id is None and be in ("rccl", "auto") and torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
        device_id = local
    if device_id is not None and torch.cuda.is_available():
        torch.cuda.set_device(device_id)
    pg = ProcessGroup(store, "pg0", rank, world_size, be, timeout_ms, list(range(world_size)), device_id)
    _state["default"] = pg
    _state["groups"] = [pg]
    _state["group_count"] = 1
    GroupMember.WORLD = pg
    if be == "rccl" and device_id is not None:
        pg.rccl_comm(device_id)  # eager init: fail fast on RCCL problems


def destroy_process_group(group=None) -> None:
    if group is not None and group is not get_default_group():
        if group in _state["groups"]:
            _state["groups"].remove(group)
        group._host = None
        group._rccl = None
        return
    pg = _state["default"]
    if pg is None:
        return
    # Rendezvous before tearing the store server (rank 0) down.
    try:
        pg.store.barrier("destroy")
    except Exception:
        pass
    for g in _state["groups"]:
        g._host = None
        g._rccl = None
    _state["default"] = None
    _state["groups"] = []
    GroupMember.WORLD = None


def get_rank(group=None) -> int:
    if group is None and not is_initialized():
        return 0
    return _group(group).rank()


def get_world_size(group=None) -> int:
    if group is None and not is_initialized():
        return 1
    return _group(group).size()


def get_backend(group=None) -> str:
    return _group(group).backend


def new_group(ranks: Optional[List[int]] = None, timeout=None, backend=None, pg_options=None):
    """Collective over the default group: every rank must call it (torch
    semantics). On RCCL the sub-communicator comes from ``ncclCommSplit`` of
    the world communicator (every rank joins the split; non-members pass
    NOCOLOR) — no second unique-id rendezvous and the parent's xGMI topology
    is reused. The host backend builds its group communicator lazily through
    the store."""
    world = get_default_group()
    ranks = sorted(range(world.size()) if ranks is None else ranks)
    _state["group_count"] += 1
    prefix = f"pg{_state['group_count'] - 1}"
    member = world.rank() in ranks
    be = _BACKEND_ALIASES.get((backend or world.backend).lower(), world.backend)
    sub = None
    if be in ("rccl", "auto") and world._rccl is not None:
        sub = world._rccl.split(0 if member else -1, ranks.index(world.rank()) if member else 0, prefix)
    if not member:
        return GroupMember.NON_GROUP_MEMBER
    tms = int(timeout.total_seconds() * 1000) if timeout else world.timeout_ms
    pg = ProcessGroup(world.store, prefix, ranks.index(world.rank()), len(ranks), be, tms, ranks, world.device_id)
    if sub is not None:
        pg._rccl = sub
    _state["groups"].append(pg)
    return pg


def _ret(work, async_op):
    if async_op:
        return work
    work.wait()
    return None


def all_reduce(tensor: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    pg = _group(group)
    return _ret(pg.comm_for(tensor).all_reduce(tensor, _to_op(op)), async_op)


def broadcast(tensor: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    pg = _group(group)
    root = pg.global_ranks.index(src) if group is not None and group is not GroupMember.WORLD else src
    return _ret(pg.comm_for(tensor).broadcast(tensor, root), async_op)


def all_gather_into_tensor(output_tensor, input_tensor, group=None, async_op=False):
    pg = _group(group)
    return _ret(pg.comm_for(input_tensor).all_gather(output_tensor, input_tensor.contiguous()), async_op)


class _ScatterBackWork:
    """Work of a list-form all_gather: ``wait()`` orders the caller after the
    gather, then copies the rows out (on the device stream: no host block)."""

    def __init__(self, work, flat, outs):
        self._w, self._flat, self._outs, self._done = work, flat, outs, False

    def is_completed(self):
        return self._w.is_completed()

    def wait(self):
        self._w.wait()
        if not self._done:
            self._done = True
            for i, t in enumerate(self._outs):
                t.copy_(self._flat[i])
        return True

    def synchronize(self):
        self.wait()
        self._w.synchronize()


def all_gather(tensor_list: List[torch.Tensor], tensor: torch.Tensor, group=None, async_op=False):
    pg = _group(group)
    flat = torch.empty((pg.size(),) + tuple(tensor.shape), dtype=tensor.dtype, device=tensor.device)
    w = _ScatterBackWork(pg.comm_for(tensor).all_gather(flat, tensor.contiguous()), flat, tensor_list)
    if async_op:
        return w
    w.wait()
    return None


def reduce_scatter_tensor(output, input, op=ReduceOp.SUM, group=None, async_op=False):
    pg = _group(group)
    return _ret(pg.comm_for(input).reduce_scatter(output, input.contiguous(), _to_op(op)), async_op)


def reduce_scatter(output, input_list, op=ReduceOp.SUM, group=None, async_op=False):
    flat = torch.cat([t.reshape(-1) for t in input_list])
    return reduce_scatter_tensor(output, flat, op, group, async_op)


def all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, group=None,
                      async_op=False):
    if output_split_sizes or input_split_sizes:
        raise NotImplementedError("uneven all_to_all splits are not supported")
    pg = _group(group)
    return _ret(pg.comm_for(input).all_to_all(output, input.contiguous()), async_op)


def _peer(pg, r, group):
    return pg.global_ranks.index(r) if group is not None and group is not GroupMember.WORLD else r


def isend(tensor, dst, group=None, tag=0):
    pg = _group(group)
    return pg.comm_for(tensor).send(tensor.contiguous(), _peer(pg, dst, group))


def irecv(tensor, src, group=None, tag=0):
    pg = _group(group)
    return pg.comm_for(tensor).recv(tensor, _peer(pg, src, group))


def send(tensor, dst, group=None, tag=0):
    isend(tensor, dst, group, tag).wait()


def recv(tensor, src, group=None, tag=0):
    irecv(tensor, src, group, tag).wait()
    return src


def barrier(group=None, async_op=False, device_ids=None):
    pg = _group(group)
    if pg.backend in ("rccl", "auto") and torch.cuda.is_available() and pg.device_id is not None:
        w = pg.rccl_comm().barrier()
    else:
        w = pg.host_comm().barrier()
        w.wait()
    return w if async_op else None


# Object collectives ride on the store (rank-local pickles of this program's
# own objects; nothing external is ever unpickled). The call sequence number is
# per group: only the group's members call its object collectives, so a world
# counter would drift between members and non-members after a sub-group call
# and the next world-level call would read different keys on different ranks.
# Every rank counts its reads done; the last reader deletes the call's keys.


def _obj_key(pg, kind):
    n = pg._obj_seq
    pg._obj_seq += 1
    return f"{pg.prefix}/obj/{kind}/{n}"


def _obj_release(pg, keys, base):
    if pg.store.add(f"{base}/done", 1) == pg.size():
        for k in (*keys, f"{base}/done"):
            pg.store.delete_key(k)


def broadcast_object_list(object_list, src=0, group=None, device=None):
    pg = _group(group)
    key = _obj_key(pg, "bcast")
    if pg.global_ranks[pg.rank()] == src:
        pg.store.set(key, pickle.dumps(list(object_list)))
    data = pickle.loads(pg.store.get(key))
    for i, o in enumerate(data):
        object_list[i] = o
    _obj_release(pg, [key], key)


def all_gather_object(object_list, obj, group=None):
    pg = _group(group)
    base = _obj_key(pg, "gather")
    pg.store.set(f"{base}/{pg.rank()}", pickle.dumps(obj))
    keys = [f"{base}/{r}" for r in range(pg.size())]
    for r, k in enumerate(keys):
        object_list[r] = pickle.loads(pg.store.get(k))
    _obj_release(pg, keys, base)


from . import launch  # noqa: E402,F401  (spawn / launch_env / free_port)
from .launch import spawn  # noqa: E402,F401
