"""Micro-step weight-gradient deferral (DistributedDataParallel(
defer_accum_wgrad=True), ops/linear.py): under no_sync the Linear weight
gradients are kept as (dY, X) row segments and the synchronising micro-step
computes each over all micro-steps in one multi-segment wgrad launch. The
gradients must equal the per-micro-step accumulation (fp32 summation order
aside), and nothing may be lost when no synchronising backward follows
(the optimizer step flushes)."""
import contextlib
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(cuda):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    yield
    dcp.distributed.destroy_process_group()


@pytest.fixture
def no_autotune():
    from distributed_compute_pytorch_amd.ops import linear as lin

    old = lin._AUTOTUNE
    lin._AUTOTUNE = False  # both arms on the same kernels: only the deferral differs
    yield
    lin._AUTOTUNE = old


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _model(cuda):
    from distributed_compute_pytorch_amd import models

    torch.manual_seed(0)
    return models.gpt2_small(n_layer=2, dropout=0.0, fused=True).to(cuda)


def _grads(base, data, defer, cuda, sync_last=True):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.ops import linear as lin

    m = copy.deepcopy(base)
    ddp = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True,
                                               defer_accum_wgrad=defer)
    pending = []
    for k, seq in enumerate(data):
        last = sync_last and k == len(data) - 1
        with (contextlib.nullcontext() if last else ddp.no_sync()):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ddp(seq[:, :-1], seq[:, 1:]) / len(data)
            loss.backward()
        pending.append(lin.pending_weight_grads())
    torch.cuda.synchronize()
    return m, ddp, pending


def test_deferred_wgrad_matches_per_microstep(pg, cuda, no_autotune):
    from distributed_compute_pytorch_amd.ops import linear as lin

    base = _model(cuda)
    data = [torch.randint(0, 50257, (2, 513), device=cuda) for _ in range(4)]  # 1,024 rows per micro-step
    m_ref, _, p_ref = _grads(base, data, False, cuda)
    m_def, _, p_def = _grads(base, data, True, cuda)
    assert p_ref == [0, 0, 0, 0]
    assert p_def[0] > 0 and p_def[1] == p_def[0] and p_def[-1] == 0  # stashed, then consumed
    n_lin = 0
    for (name, a), b in zip(m_ref.named_parameters(), m_def.parameters()):
        assert b.grad is not None, name
        assert _rel(b.grad, a.grad) < 1e-4, (name, _rel(b.grad, a.grad))
        n_lin += a.dim() == 2 and "wte" not in name and "wpe" not in name
    assert n_lin >= 8  # the Linear weights were covered
    assert lin.pending_weight_grads() == 0


def test_optimizer_step_flushes_deferred(pg, cuda, no_autotune):
    """no_sync micro-steps only, then a stock torch.optim step: the global step
    pre-hook adds the deferred contributions before the update."""
    from distributed_compute_pytorch_amd.ops import linear as lin

    base = _model(cuda)
    data = [torch.randint(0, 50257, (2, 257), device=cuda) for _ in range(2)]
    m_ref, _, _ = _grads(base, data, False, cuda, sync_last=False)
    m_def, _, pend = _grads(base, data, True, cuda, sync_last=False)
    assert pend[-1] > 0
    opt = torch.optim.SGD(m_def.parameters(), lr=0.0)  # lr 0: only the flush is observed
    opt.step()
    assert lin.pending_weight_grads() == 0
    for (name, a), b in zip(m_ref.named_parameters(), m_def.parameters()):
        assert b.grad is not None, name
        assert _rel(b.grad, a.grad) < 1e-4, (name, _rel(b.grad, a.grad))


def test_wgrad_multi_segments_match_fp64(cuda):
    """The multi-segment launch itself: ragged segment lengths (each padded to
    whole K-tiles), 1-4 segments, accumulation into an existing gradient."""
    from distributed_compute_pytorch_amd._ext import C as _C

    g = torch.Generator().manual_seed(21)
    n1, n2 = 768, 512
    rows = [1000, 640, 2049, 64]
    gys = [torch.randn(r, n1, generator=g).to(torch.bfloat16).to(cuda) for r in rows]
    xs = [torch.randn(r, n2, generator=g).to(torch.bfloat16).to(cuda) for r in rows]
    for k in range(1, 5):
        ref = sum(a.double().t() @ b.double() for a, b in zip(gys[:k], xs[:k]))
        dw = _C.conv1x1_wgrad_multi(gys[:k], xs[:k])
        assert _rel(dw, ref) < 1e-5, k
        base = torch.randn(n1, n2, generator=g).to(cuda)
        acc = base.clone()
        _C.conv1x1_wgrad_multi(gys[:k], xs[:k], accumulate_into=acc)
        assert _rel(acc, ref + base.double()) < 1e-5, k


def test_colsum_multi_matches_fp64(cuda):
    """The deferred bias gradient's one-launch column sum over 1-4 row
    segments of different lengths, fresh and accumulating."""
    from distributed_compute_pytorch_amd._ext import C as _C

    g = torch.Generator().manual_seed(22)
    n = 2304
    segs = [torch.randn(r, n, generator=g).to(torch.bfloat16).to(cuda) for r in (8192, 1000, 3, 4097)]
    for k in range(1, 5):
        ref = sum(s.double().sum(0) for s in segs[:k])
        out = _C.colsum_multi(segs[:k])
        assert _rel(out, ref) < 1e-5, k
        base = torch.randn(n, generator=g).to(cuda)
        acc = base.clone()
        _C.colsum_multi(segs[:k], accumulate_into=acc)
        assert _rel(acc, ref + base.double()) < 1e-5, k
    # the single-segment colsum (same kernel) still agrees
    assert _rel(_C.colsum(segs[0]), segs[0].double().sum(0)) < 1e-5


def test_zero_grad_drops_deferred(pg, cuda, no_autotune):
    """zero_grad of a fused optimizer after no_sync micro-steps (a skipped
    step): the stashed contributions go with .grad — the next accumulation
    round's gradients equal a fresh run's."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.ops import linear as lin

    base = _model(cuda)
    data = [torch.randint(0, 50257, (2, 257), device=cuda) for _ in range(2)]
    m_ref, _, _ = _grads(base, data, True, cuda)
    m = copy.deepcopy(base)
    ddp = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True, defer_accum_wgrad=True)
    opt = dcp.optim.SGD(m.parameters(), lr=0.0)
    with ddp.no_sync():  # an accumulation round that is abandoned
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ddp(data[1][:, :-1], data[1][:, 1:]).backward()
    assert lin.pending_weight_grads() > 0
    opt.zero_grad(set_to_none=True)
    assert lin.pending_weight_grads() == 0
    for k, seq in enumerate(data):
        with (contextlib.nullcontext() if k == len(data) - 1 else ddp.no_sync()):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ddp(seq[:, :-1], seq[:, 1:]) / len(data)
            loss.backward()
    torch.cuda.synchronize()
    for (name, a), b in zip(m_ref.named_parameters(), m.parameters()):
        assert _rel(b.grad, a.grad) < 1e-4, (name, _rel(b.grad, a.grad))


@pytest.mark.parametrize("how", ["module", "stock_optimizer"])
def test_stock_zero_grad_drops_deferred(pg, cuda, no_autotune, how):
    """a stock zero_grad (torch's Module / Optimizer, no hooks of
    their own) abandoning an accumulation round drops the stashed micro-steps
    too — the next round's gradients equal a fresh run's."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.ops import linear as lin

    base = _model(cuda)
    data = [torch.randint(0, 50257, (2, 257), device=cuda) for _ in range(2)]
    m_ref, _, _ = _grads(base, data, True, cuda)
    m = copy.deepcopy(base)
    ddp = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True, defer_accum_wgrad=True)
    with ddp.no_sync():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ddp(data[1][:, :-1], data[1][:, 1:]).backward()
    assert lin.pending_weight_grads() > 0
    if how == "module":
        ddp.zero_grad()
    else:
        torch.optim.SGD(m.parameters(), lr=0.0).zero_grad()
    assert lin.pending_weight_grads() == 0
    for k, seq in enumerate(data):
        with (contextlib.nullcontext() if k == len(data) - 1 else ddp.no_sync()):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ddp(seq[:, :-1], seq[:, 1:]) / len(data)
            loss.backward()
    torch.cuda.synchronize()
    for (name, a), b in zip(m_ref.named_parameters(), m.parameters()):
        assert _rel(b.grad, a.grad) < 1e-4, (name, _rel(b.grad, a.grad))


class _TwoBranch(torch.nn.Module):
    """Linear ``a`` always runs; ``b`` only when asked (a branch the
    synchronising micro-step may skip)."""

    def __init__(self):
        super().__init__()
        from distributed_compute_pytorch_amd.ops.linear import FusedLinear

        self.a = FusedLinear(256, 512)
        self.b = FusedLinear(256, 512)

    def forward(self, x, use_b=True):
        y = self.a(x).float().square().sum() * 1e-4  # (sum: an empty micro-batch gives 0, not NaN)
        if use_b:
            y = y + self.b(x).float().square().sum() * 1e-4
        return y


def _two_branch_grads(base, xs, use_b, defer):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.ops import linear as lin

    m = copy.deepcopy(base)
    ddp = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True,
                                               find_unused_parameters=True, defer_accum_wgrad=defer)
    for k, (x, ub) in enumerate(zip(xs, use_b)):
        with (contextlib.nullcontext() if k == len(xs) - 1 else ddp.no_sync()):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ddp(x, ub)
            loss.backward()
    torch.cuda.synchronize()
    # right after the synchronised backward (no optimizer step): nothing may
    # be left for a post-reduction flush
    assert lin.pending_weight_grads() == 0
    return m


def test_deferred_segments_of_skipped_linear_join_the_reduction(pg, cuda, no_autotune):
    """a Linear that runs under no_sync but not in the synchronising
    micro-step must have its stashed contributions in .grad before the bucket
    reduction (not added unreduced at the optimizer step)."""
    torch.manual_seed(3)
    base = _TwoBranch().to(cuda)
    xs = [torch.randn(512, 256, device=cuda) for _ in range(3)]
    use_b = [True, True, False]
    ref = _two_branch_grads(base, xs, use_b, False)
    got = _two_branch_grads(base, xs, use_b, True)
    for (name, a), b in zip(ref.named_parameters(), got.parameters()):
        assert b.grad is not None, name
        assert _rel(b.grad, a.grad) < 1e-4, (name, _rel(b.grad, a.grad))


def test_deferred_segments_with_empty_sync_microbatch(pg, cuda, no_autotune):
    """An empty synchronising micro-batch still consumes the stashed segments."""
    torch.manual_seed(4)
    base = _TwoBranch().to(cuda)
    xs = [torch.randn(384, 256, device=cuda), torch.randn(640, 256, device=cuda), torch.randn(0, 256, device=cuda)]
    use_b = [True, True, True]
    ref = _two_branch_grads(base, xs, use_b, False)
    got = _two_branch_grads(base, xs, use_b, True)
    for (name, a), b in zip(ref.named_parameters(), got.parameters()):
        assert b.grad is not None, name
        assert _rel(b.grad, a.grad) < 1e-4, (name, _rel(b.grad, a.grad))
