"""DDP parity oracle on CPU: our DDP (host backend) vs stock torch DDP (gloo),
world_size 2, same model / seeds / data (SURVEY §4.2 'Integration parity oracle')."""
import copy
import datetime
import os

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from mp_util import run_world


def _init_torch_pg(rank, world):
    import torch.distributed as tdist

    port = int(os.environ["DCP_TEST_TORCH_PORT"])  # picked free by run_world
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                             timeout=datetime.timedelta(seconds=60))
    return tdist


def _step(model, opt, x, y, seed):
    opt.zero_grad()
    with torch.random.fork_rng():
        torch.manual_seed(seed)
        loss = F.nll_loss(model(x), y)
    loss.backward()
    opt.step()
    return loss.detach()


def _parity(rank, world, kwargs, steps, accumulate):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet

    tdist = _init_torch_pg(rank, world)
    torch.manual_seed(0)
    m_ours = ConvNet()
    m_ref = copy.deepcopy(m_ours)
    ours = dcp.parallel.DistributedDataParallel(m_ours, **kwargs)
    ref_kw = {k: v for k, v in kwargs.items() if k in ("gradient_as_bucket_view", "bucket_cap_mb",
                                                         "find_unused_parameters", "broadcast_buffers")}
    ref = nn.parallel.DistributedDataParallel(m_ref, **ref_kw)
    o1 = dcp.optim.Adadelta(ours.parameters(), lr=1e-3)
    o2 = torch.optim.Adadelta(ref.parameters(), lr=1e-3)
    s1 = dcp.optim.StepLR(o1, step_size=1, gamma=0.7)
    s2 = torch.optim.lr_scheduler.StepLR(o2, step_size=1, gamma=0.7)
    g = torch.Generator().manual_seed(100 + rank)
    for it in range(steps):
        xs = [torch.randn(16, 1, 28, 28, generator=g) for _ in range(accumulate)]
        ys = [torch.randint(0, 10, (16,), generator=g) for _ in range(accumulate)]
        losses = []
        for model, opt in ((ours, o1), (ref, o2)):
            opt.zero_grad()
            for k in range(accumulate):
                ctx = model.no_sync() if k < accumulate - 1 else _null()
                with ctx:
                    with torch.random.fork_rng():
                        torch.manual_seed(1000 * it + k)
                        loss = F.nll_loss(model(xs[k]), ys[k])
                    loss.backward()
            opt.step()
            losses.append(loss.detach())
        torch.testing.assert_close(losses[0], losses[1], rtol=1e-5, atol=1e-6)
        s1.step()
        s2.step()
    for (n, p), q in zip(m_ref.named_parameters(), m_ours.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-5, atol=1e-6, msg=n)
    for (n, b), c in zip(m_ref.named_buffers(), m_ours.buffers()):
        torch.testing.assert_close(c, b, rtol=2e-5, atol=1e-6, msg=n)
    assert list(ours.state_dict().keys()) == list(ref.state_dict().keys())
    assert o1.state_dict()["param_groups"][0]["lr"] == pytest.approx(o2.state_dict()["param_groups"][0]["lr"])
    assert list(o1.state_dict()["state"][0].keys()) == list(o2.state_dict()["state"][0].keys())
    # all ranks hold identical replicas
    flat = torch.cat([p.detach().reshape(-1) for p in m_ours.parameters()])
    other = flat.clone()
    dcp.distributed.broadcast(other, 0)
    torch.testing.assert_close(flat, other)
    tdist.destroy_process_group()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


@pytest.mark.parametrize("kwargs", [{}, {"gradient_as_bucket_view": True}, {"bucket_cap_mb": 0.05},
                                    {"broadcast_buffers": False},
                                    {"gradient_as_bucket_view": True, "bucket_cap_mb": 0.05,
                                     "overlap_optimizer": True}])
def test_ddp_matches_torch_ddp(kwargs):
    run_world(_parity, 2, kwargs, 3, 1)


def _overlap(rank, world):
    """overlap_optimizer: after backward the bucket reductions stay deferred
    (fc1.weight, 4.7 MB, is a bucket far over the 0.05 MB cap); the fused
    optimizer syncs them bucket by bucket; results equal the non-overlapped
    DDP bit for bit, and nothing is left deferred after the step."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet

    torch.manual_seed(0)
    base = ConvNet()
    runs = {}
    for ov in (False, True):
        m = copy.deepcopy(base)
        ddp = dcp.parallel.DistributedDataParallel(m, gradient_as_bucket_view=True, bucket_cap_mb=0.05,
                                                   overlap_optimizer=ov)
        opt = dcp.optim.Adadelta(ddp.parameters(), lr=1e-2)
        g = torch.Generator().manual_seed(7 + rank)
        deferred = []
        for it in range(4):
            opt.zero_grad(set_to_none=True)
            x, y = torch.randn(8, 1, 28, 28, generator=g), torch.randint(0, 10, (8,), generator=g)
            with torch.random.fork_rng():
                torch.manual_seed(it)
                F.nll_loss(ddp(x), y).backward()
            deferred.append(len(ddp.reducer.deferred_buckets()))
            opt.step()
            assert ddp.reducer.deferred_buckets() == []
        if ov:
            nb = len(ddp.bucket_sizes())
            assert deferred[0] == 0 and all(d == nb for d in deferred[1:]), (deferred, nb)
            assert max(ddp.bucket_sizes()) > 0.05 * 2**20
        else:
            assert deferred == [0] * 4
        runs[ov] = [p.detach().clone() for p in m.parameters()]
    for a, b in zip(runs[False], runs[True]):
        assert torch.equal(a, b)


def test_overlap_optimizer_defers_and_matches():
    run_world(_overlap, 2)


def _overlap_stock(rank, world):
    """overlap_optimizer with STOCK consumers of .grad:
    torch.nn.utils.clip_grad_norm_ and torch.optim.AdamW read the gradients
    while the bucket reductions are deferred. The pending views must order
    them behind the reductions: parameters equal the non-overlapped run bit
    for bit, and the gradients handed out after backward are the pending
    wrappers (nothing else reads a buffer mid-reduction)."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet
    from distributed_compute_pytorch_amd.parallel.ddp import _PendingGrad

    torch.manual_seed(0)
    base = ConvNet()
    runs = {}
    for ov in (False, True):
        m = copy.deepcopy(base)
        ddp = dcp.parallel.DistributedDataParallel(m, gradient_as_bucket_view=True, bucket_cap_mb=0.05,
                                                   overlap_optimizer=ov)
        opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3, weight_decay=0.01)
        g = torch.Generator().manual_seed(7 + rank)
        kinds = []
        for it in range(4):
            opt.zero_grad(set_to_none=True)
            x, y = torch.randn(8, 1, 28, 28, generator=g), torch.randint(0, 10, (8,), generator=g)
            with torch.random.fork_rng():
                torch.manual_seed(it)
                (F.nll_loss(ddp(x), y) * 100.0).backward()
            kinds.append(sum(isinstance(p.grad, _PendingGrad) for p in m.parameters()))
            torch.nn.utils.clip_grad_norm_(ddp.parameters(), 1.0)
            assert not any(isinstance(p.grad, _PendingGrad) for p in m.parameters())
            opt.step()
            assert ddp.reducer.deferred_buckets() == []
        if ov:
            assert kinds[0] == 0 and all(k == len(list(m.parameters())) for k in kinds[1:]), kinds
        else:
            assert kinds == [0] * 4
        runs[ov] = [p.detach().clone() for p in m.parameters()]
    for a, b in zip(runs[False], runs[True]):
        assert torch.equal(a, b)


def test_overlap_optimizer_safe_for_stock_consumers():
    run_world(_overlap_stock, 2)


def test_ddp_no_sync_accumulation_matches_torch():
    run_world(_parity, 2, {}, 2, 3)


def _bucket_rebuild(rank, world):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet

    torch.manual_seed(0)
    m = dcp.parallel.DistributedDataParallel(ConvNet())
    x = torch.randn(4, 1, 28, 28)
    for _ in range(2):
        F.nll_loss(m(x), torch.zeros(4, dtype=torch.long)).backward()
    info = m.ddp_logging_data()
    # torch rebuilds into 4,725,288 B + 75,264 B
    assert info["bucket_sizes"] == [4725288, 75264], info
    assert info["rebuilds"] == 1


def test_bucket_rebuild_matches_reference_sizes():
    run_world(_bucket_rebuild, 2)


class _Branchy(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(8, 8)
        self.b = nn.Linear(8, 8)
        self.head = nn.Linear(8, 2)

    def forward(self, x, use_b):
        h = self.a(x)
        if use_b:
            h = self.b(h)
        return self.head(h)


def _unused(rank, world):
    import distributed_compute_pytorch_amd as dcp

    torch.manual_seed(0)
    m = _Branchy()
    ref = copy.deepcopy(m)
    ddp = dcp.parallel.DistributedDataParallel(m, find_unused_parameters=True)
    x = torch.randn(4, 8) + rank
    # rank 0 uses branch b, rank 1 does not: b's grad must still be averaged
    ddp(x, use_b=(rank == 0)).sum().backward()
    grads = {n: p.grad.clone() if p.grad is not None else None for n, p in m.named_parameters()}
    # expected: average of per-rank local grads (zeros for unused)
    outs = []
    for r in range(world):
        rr = copy.deepcopy(ref)
        rr(torch.randn(4, 8) * 0 + x - rank + r, use_b=(r == 0)).sum().backward()
        outs.append({n: (p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in rr.named_parameters()})
    for n in grads:
        exp = sum(o[n] for o in outs) / world
        torch.testing.assert_close(grads[n], exp, rtol=1e-5, atol=1e-6, msg=n)


def test_find_unused_parameters():
    run_world(_unused, 2)


def _unused_error(rank, world):
    import distributed_compute_pytorch_amd as dcp

    m = _Branchy()
    ddp = dcp.parallel.DistributedDataParallel(m)
    with pytest.raises(RuntimeError, match="find_unused_parameters"):
        ddp(torch.randn(2, 8), use_b=False).sum().backward()


def test_unused_without_flag_raises():
    run_world(_unused_error, 2)


def _compress(rank, world):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.parallel import comm_hooks

    torch.manual_seed(0)
    base = nn.Sequential(nn.Linear(32, 64), nn.ReLU(), nn.Linear(64, 4))
    a, b, c = copy.deepcopy(base), copy.deepcopy(base), copy.deepcopy(base)
    da = dcp.parallel.DistributedDataParallel(a)
    db = dcp.parallel.DistributedDataParallel(b, comm_dtype=torch.bfloat16)
    dc = dcp.parallel.DistributedDataParallel(c)
    dc.register_comm_hook(None, comm_hooks.allreduce_hook)
    x = torch.randn(8, 32) * (rank + 1)
    for d in (da, db, dc):
        d(x).pow(2).sum().backward()
    for pa, pb, pc in zip(a.parameters(), b.parameters(), c.parameters()):
        torch.testing.assert_close(pc.grad, pa.grad)
        torch.testing.assert_close(pb.grad, pa.grad, rtol=2e-2, atol=2e-2)


def test_bf16_wire_compression_and_comm_hook():
    run_world(_compress, 2)


def _ckpt(rank, world, path):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet

    torch.manual_seed(0)
    m = dcp.parallel.DistributedDataParallel(ConvNet())
    opt = dcp.optim.Adadelta(m.parameters(), lr=1e-3)
    sch = dcp.optim.StepLR(opt, 1, 0.7)
    F.nll_loss(m(torch.randn(4, 1, 28, 28)), torch.zeros(4, dtype=torch.long)).backward()
    opt.step()
    sch.step()
    dcp.utils.save_checkpoint(path, m, opt, sch, epoch=3, step=7)
    dcp.utils.save_model(m, path + ".model")
    m2 = dcp.parallel.DistributedDataParallel(ConvNet())
    opt2 = dcp.optim.Adadelta(m2.parameters(), lr=1e-3)
    sch2 = dcp.optim.StepLR(opt2, 1, 0.7)
    meta = dcp.utils.load_checkpoint(path, m2, opt2, sch2)
    assert meta["epoch"] == 3 and meta["step"] == 7
    for p, q in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q)
    assert opt2.param_groups[0]["lr"] == pytest.approx(0.7e-3)
    sd = torch.load(path + ".model", weights_only=True)
    assert next(iter(sd)).startswith("module.")
    from distributed_compute_pytorch_amd.models import ConvNet as CN
    plain = CN()
    plain.load_state_dict({k[len("module."):]: v for k, v in sd.items()})


def test_checkpoint_roundtrip(tmp_path):
    run_world(_ckpt, 2, str(tmp_path / "ck.pt"))


class _TinyLM(nn.Module):
    """Transformer-shaped: an embedding past the 16 MiB bucket cap (one
    parameter larger than a bucket, tied to the output head, ready last),
    LayerNorm + MLP blocks."""

    def __init__(self, vocab=70000, d=64, layers=2):
        super().__init__()
        self.emb = nn.Embedding(vocab, d)
        self.blocks = nn.ModuleList(nn.Sequential(nn.LayerNorm(d), nn.Linear(d, 4 * d), nn.GELU(), nn.Linear(4 * d, d))
                                    for _ in range(layers))
        self.ln = nn.LayerNorm(d)

    def forward(self, idx, tgt):
        h = self.emb(idx)
        for b in self.blocks:
            h = h + b(h)
        logits = self.ln(h) @ self.emb.weight.t()
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]), tgt.reshape(-1))


def _tiny_lm_parity(rank, world):
    """ws=4: our DDP with the xGMI bucket plan (16 MiB cap, 1 MiB first, 2 MiB
    tail), gradient-as-bucket-view and overlap_optimizer against torch gloo
    DDP (same cap), both stepping torch.optim.AdamW; 2 micro-steps of
    gradient accumulation (no_sync) per step, 3 steps."""
    import distributed_compute_pytorch_amd as dcp

    tdist = _init_torch_pg(rank, world)
    torch.manual_seed(0)
    m_ours = _TinyLM()
    m_ref = copy.deepcopy(m_ours)
    assert m_ours.emb.weight.numel() * 4 > dcp.parallel.XGMI_BUCKETS["bucket_cap_mb"] * 2**20
    ours = dcp.parallel.DistributedDataParallel(m_ours, gradient_as_bucket_view=True, overlap_optimizer=True,
                                                **dcp.parallel.XGMI_BUCKETS)
    ref = nn.parallel.DistributedDataParallel(m_ref, gradient_as_bucket_view=True, bucket_cap_mb=16)
    o1 = torch.optim.AdamW(ours.parameters(), lr=1e-3, weight_decay=0.01)
    o2 = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.01)
    g = torch.Generator().manual_seed(50 + rank)
    for it in range(3):
        batches = [(torch.randint(0, 70000, (4, 16), generator=g), torch.randint(0, 70000, (4, 16), generator=g))
                   for _ in range(2)]
        losses = []
        for model, opt in ((ours, o1), (ref, o2)):
            opt.zero_grad(set_to_none=True)
            for k, (x, y) in enumerate(batches):
                with (model.no_sync() if k == 0 else _null()):
                    loss = model(x, y) / 2
                    loss.backward()
            opt.step()
            losses.append(loss.detach())
        torch.testing.assert_close(losses[0], losses[1], rtol=1e-5, atol=1e-6)
    for (n, p), q in zip(m_ref.named_parameters(), m_ours.parameters()):
        torch.testing.assert_close(q, p, rtol=1e-5, atol=1e-6, msg=n)
    sizes = ours.bucket_sizes()
    assert len(sizes) >= 2 and max(sizes) > 16 * 2**20  # the over-cap embedding bucket + the rest
    tdist.destroy_process_group()


def test_transformer_shaped_ws4_xgmi_plan_overlap_matches_torch():
    run_world(_tiny_lm_parity, 4, timeout=300)


class _BNNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(1, 8, 3)
        self.bn = nn.BatchNorm2d(8)
        self.fc = nn.Linear(8, 10)

    def forward(self, x):
        return F.log_softmax(self.fc(F.relu(self.bn(self.conv(x))).mean((2, 3))), 1)


def _buffer_sync(rank, world, overlap):
    """BatchNorm running statistics under the per-forward buffer broadcast:
    ours (broadcast started after each synchronising forward and completed at
    the next one, or torch's start-of-forward broadcast) against torch DDP —
    every rank's eval outputs and buffers after a mix of training, no_sync and
    eval forwards."""
    import distributed_compute_pytorch_amd as dcp

    tdist = _init_torch_pg(rank, world)
    torch.manual_seed(0)
    m_ours = _BNNet()
    m_ref = copy.deepcopy(m_ours)
    ours = dcp.parallel.DistributedDataParallel(m_ours, overlap_buffer_sync=overlap)
    ref = nn.parallel.DistributedDataParallel(m_ref)
    o1 = dcp.optim.SGD(ours.parameters(), lr=0.1)
    o2 = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(50 + rank)
    xe = torch.randn(4, 1, 12, 12, generator=torch.Generator().manual_seed(99))
    for it in range(4):
        x = [torch.randn(6, 1, 12, 12, generator=g) * (1 + rank) for _ in range(2)]
        y = [torch.randint(0, 10, (6,), generator=g) for _ in range(2)]
        for model, opt in ((ours, o1), (ref, o2)):
            model.train()
            opt.zero_grad()
            if it % 2:  # an accumulation step: the no_sync forward broadcasts too (torch semantics)
                with model.no_sync():
                    F.nll_loss(model(x[1]), y[1]).backward()
            F.nll_loss(model(x[0]), y[0]).backward()
            opt.step()
        if it >= 2:  # eval forwards: rank 0's statistics on every rank
            outs = []
            for model in (ours, ref):
                model.eval()
                with torch.no_grad():
                    outs.append(model(xe))
            torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-6)
            for (n, b), c in zip(m_ref.named_buffers(), m_ours.buffers()):
                torch.testing.assert_close(c, b, rtol=1e-5, atol=1e-6, msg=n)
    ours.sync_buffers()
    tdist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_buffer_broadcast_matches_torch(overlap):
    run_world(_buffer_sync, 2, overlap)


def _static_graph(rank, world):
    """static_graph=True (torch's flag): a branch unused on every iteration is
    handled without find_unused_parameters — same gradients as torch DDP
    (static_graph=True) over several iterations; from the second iteration on
    the used map is reused (no graph traversal, no used-map collective)."""
    import distributed_compute_pytorch_amd as dcp

    tdist = _init_torch_pg(rank, world)
    torch.manual_seed(0)
    m = _Branchy()
    m_ref = copy.deepcopy(m)
    ours = dcp.parallel.DistributedDataParallel(m, static_graph=True)
    ref = nn.parallel.DistributedDataParallel(m_ref, static_graph=True)
    o1 = dcp.optim.SGD(ours.parameters(), lr=0.1)
    o2 = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(7 + rank)
    ops0 = None
    for it in range(4):
        x = torch.randn(4, 8, generator=g)
        for model, opt in ((ours, o1), (ref, o2)):
            opt.zero_grad()
            model(x, use_b=False).sum().backward()
            opt.step()
        assert ours.reducer.static_frozen
        if it == 1:
            ops0 = ours._comm.ops_issued
        elif it == 2:
            # frozen: one bucket collective per bucket, no used-map all-reduce
            assert ours._comm.ops_issued - ops0 == len(ours.bucket_sizes())
    for (n, p), q in zip(m_ref.named_parameters(), m.parameters()):
        torch.testing.assert_close(q, p, rtol=1e-5, atol=1e-6, msg=n)
    tdist.destroy_process_group()


def test_static_graph_matches_torch():
    run_world(_static_graph, 2)


def _arg_validation(rank, world):
    import warnings

    import distributed_compute_pytorch_amd as dcp

    m = _Branchy()
    with pytest.raises(ValueError, match="device_ids"):
        dcp.parallel.DistributedDataParallel(m, device_ids=[0])  # CPU module
    with pytest.raises(ValueError, match="output_device"):
        dcp.parallel.DistributedDataParallel(m, output_device="cuda:0")
    with pytest.raises(TypeError, match="dim"):
        dcp.parallel.DistributedDataParallel(m, dim="0")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        dcp.parallel.DistributedDataParallel(m, check_reduction=True, find_unused_parameters=True)
    assert any("check_reduction" in str(x.message) for x in w)
    ddp = dcp.parallel.DistributedDataParallel(m, output_device="cpu", find_unused_parameters=True)
    assert ddp.output_device == "cpu"


def test_ddp_argument_validation():
    """The constructor arguments torch accepts either act or are rejected —
    none is silently stored and ignored."""
    run_world(_arg_validation, 2)


def _buffer_load(rank, world):
    """overlap_buffer_sync: a load_state_dict between two forwards (resume) is
    not overwritten by the broadcast of rank 0's pre-load buffers still in
    flight; the collective count stays the same on every rank."""
    import distributed_compute_pytorch_amd as dcp

    torch.manual_seed(0)
    m = _BNNet()
    ddp = dcp.parallel.DistributedDataParallel(m, overlap_buffer_sync=True)
    x = torch.randn(6, 1, 12, 12) * (1 + rank)
    y = torch.randint(0, 10, (6,))
    F.nll_loss(ddp(x), y).backward()
    assert ddp._buffer_bcast.pending
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for k in sd:
        if k.endswith("running_mean"):
            sd[k].fill_(3.0)  # the "checkpoint" every rank loads
    m.load_state_dict(sd)
    ddp.eval()
    with torch.no_grad():
        ddp(x)
    for k, v in m.state_dict().items():
        if k.endswith("running_mean"):
            assert torch.all(v == 3.0), k
    ddp.sync_buffers()  # still in step: one more collective on both ranks


def test_load_state_dict_not_overwritten_by_pending_broadcast():
    run_world(_buffer_load, 2)


class _EmbNet(nn.Module):
    """A tied-embedding-like net: one big parameter (the embedding, its own
    oversize bucket) and a few mid-size ones that straddle slice bounds."""

    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(3000, 64)              # 768 KB
        self.l1 = nn.Linear(64, 700)                   # ~179 KB + bias
        self.l2 = nn.Linear(700, 300)                  # ~820 KB

    def forward(self, idx):
        h = self.emb(idx).mean(1)
        h = torch.tanh(self.l1(h))
        return F.log_softmax(self.l2(h), -1)


def _sliced(rank, world, cap_mb, slice_mb, wire=None):
    """bucket_slice_mb: oversize buckets reduced slice by slice, fused AdamW
    updating each slice's parameter ranges (and whole parameters) as the
    slice lands — bit for bit the unsliced overlap run (Adam is elementwise),
    within Adam's reduction-order sensitivity of torch DDP + torch AdamW, the
    sliced buckets really issued as several collectives, nothing left
    deferred after the step, every step counter advanced once per step
    (VERDICT r5 Next 3c)."""
    import distributed_compute_pytorch_amd as dcp

    tdist = _init_torch_pg(rank, world)
    torch.manual_seed(0)
    base = _EmbNet()
    runs, sliced = {}, []
    for sm in (0.0, slice_mb, None):
        m = copy.deepcopy(base)
        if sm is None:
            model = nn.parallel.DistributedDataParallel(m, bucket_cap_mb=cap_mb)
            opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.1)
        else:
            model = dcp.parallel.DistributedDataParallel(m, gradient_as_bucket_view=True, overlap_optimizer=True,
                                                         bucket_cap_mb=cap_mb, bucket_slice_mb=sm,
                                                         **({"comm_dtype": wire} if wire is not None else {}))
            opt = dcp.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.1)
        g = torch.Generator().manual_seed(11 + rank)
        for it in range(4):
            idx = torch.randint(0, 3000, (16, 5), generator=g)
            y = torch.randint(0, 300, (16,), generator=g)
            opt.zero_grad(set_to_none=True)
            F.nll_loss(model(idx), y).backward()
            if sm:
                ks = model.reducer.deferred_buckets()
                sliced.append(sum(len(model.reducer.bucket_slice_bounds(k)) > 2 for k in ks))
            opt.step()
            if sm is not None:
                assert model.reducer.deferred_buckets() == []
        if sm is not None:
            assert all(float(opt.state[q]["step"]) == 4.0 for q in m.parameters())
        runs[sm] = [p.detach().clone() for p in m.parameters()]
    assert sliced[0] == 0 and all(n >= 1 for n in sliced[1:]), sliced  # the first iteration is never deferred
    names = [n for n, _ in base.named_parameters()]
    for n, a, b in zip(names, runs[0.0], runs[slice_mb]):
        torch.testing.assert_close(b, a, rtol=0, atol=0, msg=n)
    if wire is None:
        for n, a, b in zip(names, runs[None], runs[slice_mb]):
            # Adam turns near-zero gradients into full-size steps: the reduction
            # order (ours vs gloo) shows at ~1e-5 on a few embedding rows
            torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-4, msg=n)
    tdist.destroy_process_group()


@pytest.mark.parametrize("cap_mb,slice_mb", [(0.25, 0.25), (4.0, 0.2)])
def test_sliced_buckets_match_torch(cap_mb, slice_mb):
    run_world(_sliced, 2, cap_mb, slice_mb)


def test_sliced_buckets_bf16_wire():
    """The same with a bf16 wire: each slice unpacks its own range of the
    compressed buffer when it is synced (bit for bit the unsliced run)."""
    run_world(_sliced, 2, 4.0, 0.2, torch.bfloat16)
