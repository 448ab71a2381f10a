"""Host (CPU) communicator collectives across processes."""
import pytest
import torch

from mp_util import run_world


def _collectives(rank, world):
    import distributed_compute_pytorch_amd.distributed as dist

    for dtype in (torch.float32, torch.float64, torch.int64, torch.bfloat16):
        t = torch.arange(13, dtype=dtype) + rank
        dist.all_reduce(t)
        exp = sum(torch.arange(13, dtype=torch.float64) + r for r in range(world))
        assert torch.allclose(t.double(), exp), (dtype, t)
    t = torch.full((7,), float(rank + 1))
    dist.all_reduce(t, dist.ReduceOp.MAX)
    assert torch.all(t == world)
    t = torch.full((7,), float(rank + 1))
    dist.all_reduce(t, dist.ReduceOp.MIN)
    assert torch.all(t == 1)
    t = torch.full((1001,), float(rank))
    dist.all_reduce(t, dist.ReduceOp.AVG)
    assert torch.allclose(t, torch.full((1001,), (world - 1) / 2))
    # reference-style scalar all-reduce (main.py:65)
    loss = torch.tensor(float(rank))
    dist.all_reduce(loss, op=dist.ReduceOp.SUM)
    assert loss.item() == sum(range(world))
    b = torch.tensor([rank * 10.0, 1.0])
    dist.broadcast(b, src=world - 1)
    assert b.tolist() == [(world - 1) * 10.0, 1.0]
    out = torch.empty(world * 3)
    dist.all_gather_into_tensor(out, torch.full((3,), float(rank)))
    assert out.tolist() == sum([[float(r)] * 3 for r in range(world)], [])
    lst = [torch.empty(2) for _ in range(world)]
    dist.all_gather(lst, torch.full((2,), float(rank)))
    assert [x[0].item() for x in lst] == [float(r) for r in range(world)]
    inp = torch.arange(world * 4, dtype=torch.float32)
    o = torch.empty(4)
    dist.reduce_scatter_tensor(o, inp)
    assert torch.allclose(o, inp[rank * 4:(rank + 1) * 4] * world)
    a2a_in = torch.tensor([rank * 100.0 + j for j in range(world)])
    a2a_out = torch.empty(world)
    dist.all_to_all_single(a2a_out, a2a_in)
    assert a2a_out.tolist() == [r * 100.0 + rank for r in range(world)]
    if world >= 2:
        if rank == 0:
            dist.send(torch.tensor([42.0]), 1)
        elif rank == 1:
            x = torch.empty(1)
            dist.recv(x, 0)
            assert x.item() == 42.0
    w = dist.all_reduce(torch.ones(3), async_op=True)
    w.wait()
    dist.barrier()
    objs = [None] * world
    dist.all_gather_object(objs, {"r": rank})
    assert objs == [{"r": r} for r in range(world)]
    ol = [rank] if rank == 0 else [None]
    dist.broadcast_object_list(ol, src=0)
    assert ol == [0]


@pytest.mark.parametrize("world", [2, 3])
def test_host_collectives(world):
    run_world(_collectives, world)


def _subgroups(rank, world):
    import distributed_compute_pytorch_amd.distributed as dist

    g = dist.new_group([0, 2])
    t = torch.tensor([float(rank)])
    if rank in (0, 2):
        dist.all_reduce(t, group=g)
        assert t.item() == 2.0
        assert dist.get_world_size(g) == 2
    else:
        assert g is dist.GroupMember.NON_GROUP_MEMBER
    dist.barrier()


def test_subgroups():
    run_world(_subgroups, 3)


def _subgroup_objects(rank, world):
    import distributed_compute_pytorch_amd.distributed as dist

    g = dist.new_group([0, 2])
    if rank in (0, 2):  # members only: their group's object sequence advances
        objs = [None, None]
        dist.all_gather_object(objs, ("sub", rank), group=g)
        assert objs == [("sub", 0), ("sub", 2)]
        ol = [rank * 7]
        dist.broadcast_object_list(ol, src=2, group=g)
        assert ol == [14]
    # the world-level object collectives afterwards must agree on their keys
    objs = [None] * world
    dist.all_gather_object(objs, rank)
    assert objs == list(range(world))
    ol = ["x"] if rank == 1 else [None]
    dist.broadcast_object_list(ol, src=1)
    assert ol == ["x"]
    dist.barrier()
    # every call's keys were deleted by its last reader (rank 0 hosts the store)
    pg = dist.get_default_group()
    assert not pg.store.check([f"pg0/obj/gather/0/{r}" for r in range(world)])
    assert not pg.store.check([f"{g.prefix}/obj/gather/0/0"]) if rank in (0, 2) else True


def test_subgroup_object_collectives_then_world():
    run_world(_subgroup_objects, 3)


def _fingerprint(rank, world):
    import datetime

    import distributed_compute_pytorch_amd.distributed as dist

    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=5))
    pg = dist.get_default_group()
    pg.host_comm().set_debug_fingerprint(True)
    dist.all_reduce(torch.ones(4))
    t = torch.ones(4 if rank == 0 else 5)
    try:
        dist.all_reduce(t)
        raise AssertionError("mismatch not detected")
    except RuntimeError as e:
        # rank 1 sees the fingerprint mismatch; rank 0 (whose check passes
        # against itself) sees its ring time out instead of hanging forever
        if rank == 1:
            assert "collective mismatch" in str(e), str(e)
    dist.destroy_process_group()


def test_debug_fingerprint_catches_mismatch():
    run_world(_fingerprint, 2, backend=None, timeout=300)


def _buffer_broadcast(rank, world):
    import distributed_compute_pytorch_amd.distributed as dist
    from distributed_compute_pytorch_amd.parallel.comm_utils import CoalescedBroadcaster

    # BatchNorm-like buffers: fp32 stats + int64 counter share one word group;
    # bf16 and a non-contiguous fp32 view ride along
    mean = torch.full((5,), float(rank))
    var = torch.arange(3, dtype=torch.float32) * (rank + 1)
    nbt = torch.tensor(7 * rank + 2**40, dtype=torch.int64)
    half = torch.full((4,), float(rank), dtype=torch.bfloat16)
    base = torch.arange(12, dtype=torch.float32).reshape(3, 4) + rank
    strided = base.t()
    bc = CoalescedBroadcaster([mean, var, nbt, half, strided])
    assert len(bc.plan) == 2, [p[1].dtype for p in bc.plan]  # fp32 words (incl. int64) + bf16
    bc(dist.get_default_group(), src=1)
    assert mean.tolist() == [1.0] * 5
    assert var.tolist() == [0.0, 2.0, 4.0]
    assert int(nbt) == 7 + 2**40
    assert half.tolist() == [1.0] * 4
    assert torch.equal(strided, (torch.arange(12, dtype=torch.float32).reshape(3, 4) + 1).t())


def test_buffer_broadcast_one_collective_per_word_group():
    run_world(_buffer_broadcast, 2)
