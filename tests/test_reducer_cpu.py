"""Reducer corner cases vs stock torch DDP (gloo, CPU, world_size 2).

* find_unused_parameters combined with no_sync accumulation: a
  parameter unused in the synced step keeps (and contributes) the gradient it
  accumulated locally; a globally unused one keeps its local gradient untouched;
* GradBucket.index() is the position within the iteration (not a running count);
* the "received no gradient" error leaves the Reducer usable;
* the xGMI tail-bucket split;
* new_group on the host backend.
"""
import copy
import datetime
import os

import pytest
import torch
from torch import nn

from mp_util import run_world


class _Branchy(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(8, 8)
        self.b = nn.Linear(8, 8)
        self.head = nn.Linear(8, 2)

    def forward(self, x, use_b):
        h = torch.tanh(self.a(x))
        if use_b:
            h = self.b(h)
        return self.head(h)


def _torch_pg(rank, world):
    import torch.distributed as tdist

    port = int(os.environ["DCP_TEST_TORCH_PORT"])  # picked free by run_world
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                             timeout=datetime.timedelta(seconds=60))
    return tdist


def _unused_accum(rank, world, grad_as_view, sync_uses_b):
    import distributed_compute_pytorch_amd as dcp

    tdist = _torch_pg(rank, world)
    torch.manual_seed(0)
    m1 = _Branchy()
    m2 = copy.deepcopy(m1)
    ours = dcp.parallel.DistributedDataParallel(m1, find_unused_parameters=True, gradient_as_bucket_view=grad_as_view)
    ref = nn.parallel.DistributedDataParallel(m2, find_unused_parameters=True, gradient_as_bucket_view=grad_as_view)
    g = torch.Generator().manual_seed(7 + rank)
    for it in range(3):
        xs = [torch.randn(4, 8, generator=g) for _ in range(2)]
        # micro-step 0 (no_sync): rank 0 uses branch b; synced micro-step 1:
        # b used by rank 1 only (sync_uses_b) or by nobody
        plan = [rank == 0, sync_uses_b and rank == 1]
        for model in (ours, ref):
            model.zero_grad(set_to_none=True)
            with model.no_sync():
                model(xs[0], use_b=plan[0]).pow(2).sum().backward()
            model(xs[1], use_b=plan[1]).pow(2).sum().backward()
        for (n, p), q in zip(m2.named_parameters(), m1.parameters()):
            if p.grad is None:
                assert q.grad is None or not q.grad.any(), (it, n)
            else:
                assert q.grad is not None, (it, n)
                torch.testing.assert_close(q.grad, p.grad, rtol=1e-5, atol=1e-6, msg=f"{it} {n}")
    tdist.destroy_process_group()


@pytest.mark.parametrize("grad_as_view", [False, True])
@pytest.mark.parametrize("sync_uses_b", [False, True])
def test_unused_params_with_no_sync_accumulation_match_torch(grad_as_view, sync_uses_b):
    run_world(_unused_accum, 2, grad_as_view, sync_uses_b)


def _hook_index(rank, world):
    import distributed_compute_pytorch_amd as dcp

    torch.manual_seed(0)
    m = nn.Sequential(*[nn.Linear(64, 64) for _ in range(6)])
    ddp = dcp.parallel.DistributedDataParallel(m, bucket_cap_mb=0.02, first_bucket_mb=0.02, tail_bucket_mb=0)
    seen = []

    def hook(state, bucket):
        seen.append((bucket.index(), bucket.is_last(), len(bucket.parameters())))
        return dcp.parallel.comm_hooks.allreduce_hook(None, bucket)

    ddp.register_comm_hook(None, hook)
    for _ in range(3):
        seen.clear()
        ddp(torch.randn(2, 64)).sum().backward()
        n = len(seen)  # (the plan may be rebuilt after the first iteration)
        assert n > 2
        assert [s[0] for s in seen] == list(range(n)), seen
        assert [s[1] for s in seen] == [False] * (n - 1) + [True]
        assert sum(s[2] for s in seen) == 12


def test_comm_hook_bucket_index_is_per_iteration():
    run_world(_hook_index, 2)


def _error_then_recover(rank, world):
    import distributed_compute_pytorch_amd as dcp

    torch.manual_seed(0)
    m = _Branchy()
    ddp = dcp.parallel.DistributedDataParallel(m)
    x = torch.randn(2, 8)
    with pytest.raises(RuntimeError, match="find_unused_parameters"):
        ddp(x, use_b=False).sum().backward()
    # the next complete iteration works and averages correctly
    for p in m.parameters():
        p.grad = None
    xr = x + rank
    ddp(xr, use_b=True).sum().backward()
    ref = copy.deepcopy(m)
    for p in ref.parameters():
        p.grad = None
    grads = []
    for r in range(world):
        rr = copy.deepcopy(ref)
        rr(x + r, use_b=True).sum().backward()
        grads.append([p.grad for p in rr.parameters()])
    for i, p in enumerate(m.parameters()):
        torch.testing.assert_close(p.grad, sum(g[i] for g in grads) / world, rtol=1e-5, atol=1e-6)


def test_reducer_usable_after_missing_grad_error():
    run_world(_error_then_recover, 2)


def test_split_tail_bucket():
    from distributed_compute_pytorch_amd._ext import C

    sizes = [100, 200, 300, 400, 50, 60]
    plan = [[5, 4], [3, 2, 1, 0]]
    assert C.split_tail_bucket(plan, sizes, 0) == plan
    assert C.split_tail_bucket(plan, sizes, 1000) == plan          # last bucket (1000 B) fits
    assert C.split_tail_bucket(plan, sizes, 350) == [[5, 4], [3, 2], [1, 0]]
    assert C.split_tail_bucket(plan, sizes, 10) == [[5, 4], [3, 2, 1], [0]]  # at least one param
    assert C.split_tail_bucket([[0]], sizes, 10) == [[0]]


def _default_plan(rank, world):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.parallel import ddp as ddp_mod

    torch.manual_seed(0)
    # ~28 MB of fp32 params in 7 layers + a small first-defined layer
    m = nn.Sequential(nn.Linear(16, 256), *[nn.Linear(1024, 1024) for _ in range(7)])
    m[0] = nn.Linear(16, 1024)
    # constructor defaults are torch's (25 MiB cap, 1 MiB first bucket, no tail split)
    plain = dcp.parallel.DistributedDataParallel(m).ddp_logging_data()
    assert plain["bucket_cap_bytes"] == 25 * 2**20 == int(ddp_mod.DEFAULT_BUCKET_CAP_MB * 2**20)
    assert plain["first_bucket_bytes"] == 2**20 and plain["tail_bucket_bytes"] == 0
    ddp = dcp.parallel.DistributedDataParallel(m, **dcp.parallel.XGMI_BUCKETS)
    info = ddp.ddp_logging_data()
    assert info["bucket_cap_bytes"] == int(dcp.parallel.XGMI_BUCKETS["bucket_cap_mb"] * 2**20)
    assert info["tail_bucket_bytes"] == int(dcp.parallel.XGMI_BUCKETS["tail_bucket_mb"] * 2**20) > 0
    # the last-launched bucket holds only the ready-last parameters and fits the tail cap
    assert info["bucket_sizes"][-1] <= info["tail_bucket_bytes"], info["bucket_sizes"]
    x = torch.randn(4, 16)
    for _ in range(2):
        ddp(x).sum().backward()
    info = ddp.ddp_logging_data()
    assert info["rebuilds"] == 1
    assert info["bucket_sizes"][-1] <= info["tail_bucket_bytes"], info["bucket_sizes"]
    assert 0 in info["bucket_indices"][-1]  # the first-defined layer's weight is ready last


def test_xgmi_default_plan_has_small_tail_bucket():
    run_world(_default_plan, 2)


def _groups(rank, world):
    import distributed_compute_pytorch_amd as dcp

    g01 = dcp.distributed.new_group([0, 1])
    g2 = dcp.distributed.new_group([2])
    if rank < 2:
        t = torch.tensor([float(rank + 1)])
        dcp.distributed.all_reduce(t, group=g01)
        assert t.item() == 3.0
        assert g2 is dcp.distributed.GroupMember.NON_GROUP_MEMBER
    else:
        assert g01 is dcp.distributed.GroupMember.NON_GROUP_MEMBER
        t = torch.tensor([5.0])
        dcp.distributed.all_reduce(t, group=g2)
        assert t.item() == 5.0
    outs = [torch.zeros(2) for _ in range(world)]
    w = dcp.distributed.all_gather(outs, torch.full((2,), float(rank)), async_op=True)
    w.wait()
    assert [o[0].item() for o in outs] == [float(r) for r in range(world)]


def test_new_group_and_async_all_gather():
    run_world(_groups, 3)


def _ordering_check(rank, world):
    """DCP_DEBUG_STREAMS=1: the Reducer's stream-ordering check passes on the
    normal path and catches a 'reduction' that never reached the buffer."""
    os.environ["DCP_DEBUG_STREAMS"] = "1"
    import distributed_compute_pytorch_amd as dcp

    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(32, 64), nn.Tanh(), nn.Linear(64, 8))
    ref = copy.deepcopy(m)
    ddp = dcp.parallel.DistributedDataParallel(m, bucket_cap_mb=0.005, first_bucket_mb=0.005, tail_bucket_mb=0)
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(4, 32, generator=g) for _ in range(world)]
    for _ in range(3):
        for p in m.parameters():
            p.grad = None
        ddp(xs[rank]).pow(2).sum().backward()
    grads = []
    for r in range(world):
        rr = copy.deepcopy(ref)
        rr(xs[r]).pow(2).sum().backward()
        grads.append([p.grad for p in rr.parameters()])
    for i, p in enumerate(m.parameters()):
        torch.testing.assert_close(p.grad, sum(gg[i] for gg in grads) / world, rtol=1e-5, atol=1e-6)
    # a comm hook whose work "completes" without reducing: ranks hold different
    # gradients, so the buffer the consumer sees is not the reduction
    ddp.register_comm_hook(None, dcp.parallel.comm_hooks.noop_hook)
    for p in m.parameters():
        p.grad = None
    with pytest.raises(RuntimeError, match="stream-ordering check failed"):
        ddp(xs[rank]).pow(2).sum().backward()


def test_reducer_stream_ordering_check():
    run_world(_ordering_check, 2)


def _compress_check(rank, world):
    """DCP_DEBUG_STREAMS=1 with the bf16 compression hook: the hook declares
    its wire precision, so its rounding is not reported as an ordering error
    (and the gradients are the bf16-rounded average)."""
    os.environ["DCP_DEBUG_STREAMS"] = "1"
    import distributed_compute_pytorch_amd as dcp

    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(32, 64), nn.Tanh(), nn.Linear(64, 8))
    ref = copy.deepcopy(m)
    ddp = dcp.parallel.DistributedDataParallel(m, bucket_cap_mb=0.005, first_bucket_mb=0.005, tail_bucket_mb=0)
    ddp.register_comm_hook(None, dcp.parallel.comm_hooks.bf16_compress_hook)
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(4, 32, generator=g) for _ in range(world)]
    for _ in range(3):
        for p in m.parameters():
            p.grad = None
        ddp(xs[rank]).pow(2).sum().backward()
    grads = []
    for r in range(world):
        rr = copy.deepcopy(ref)
        rr(xs[r]).pow(2).sum().backward()
        grads.append([p.grad for p in rr.parameters()])
    for i, p in enumerate(m.parameters()):
        torch.testing.assert_close(p.grad, sum(gg[i] for gg in grads) / world, rtol=2e-2, atol=1e-2)


def test_reducer_stream_check_tolerates_compression_hook():
    run_world(_compress_check, 2)
