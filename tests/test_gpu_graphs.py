"""Whole-step HIP-graph capture: replays must equal eager execution, and
captured ops must not depend on state outside the graph (each replay of a
captured op equals the eager op)."""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


# gemm=False runs MIOpen's stride-2 3x3 backward-weights, whose replays go
# non-finite (a stock-torch ResNet shows the same, tools/graph_nan_debug.py "r18
# plain"): its output zeroing is a captured memset node, which this ROCm does not
# order before the next kernel on replays after the first. Our kernels never
# capture memset / memcpy nodes (fused.cpp zeroed_floats, ops.cpp get_table).
@pytest.mark.parametrize("gemm", [pytest.param(False, marks=pytest.mark.xfail(
    reason="vendor: MIOpen stride-2 wgrad is not HIP-graph replay safe on this ROCm", strict=False)), True])
def test_captured_step_matches_eager(cuda, gemm):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port
    from distributed_compute_pytorch_amd.models import resnet18_like
    from distributed_compute_pytorch_amd.utils.graphs import CapturedStep, capture_stream

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    try:
        torch.manual_seed(0)
        base = resnet18_like(num_classes=10, fused_bn=True, fused_gemm=gemm).to(cuda).to(
            memory_format=torch.channels_last)
        m_eager, m_graph = copy.deepcopy(base), copy.deepcopy(base)
        d_e = dcp.parallel.DistributedDataParallel(m_eager, device_ids=[0], gradient_as_bucket_view=True)
        s = capture_stream()
        with torch.cuda.stream(s):
            d_g = dcp.parallel.DistributedDataParallel(m_graph, device_ids=[0], gradient_as_bucket_view=True)
        # small LR: a diverging run amplifies the (atomic-order) run-to-run
        # noise of the BN reductions into O(1) loss differences
        o_e = dcp.optim.SGD(d_e.parameters(), lr=0.005, momentum=0.9)
        o_g = dcp.optim.SGD(d_g.parameters(), lr=0.005, momentum=0.9)
        g = torch.Generator(device="cpu").manual_seed(1)
        batches = [(torch.randn(8, 3, 64, 64, generator=g).to(cuda).contiguous(memory_format=torch.channels_last),
                    torch.randint(0, 10, (8,), generator=g).to(cuda)) for _ in range(8)]

        def make(ddp, opt):
            def run(x, y):
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = F.cross_entropy(ddp(x), y)
                loss.backward()
                opt.step()
                return loss
            return run

        run_e, run_g = make(d_e, o_e), make(d_g, o_g)
        # the capture helper runs 3 warmup steps on the first batch
        for _ in range(3):
            run_e(*batches[0])
        cap = CapturedStep(run_g, [t.clone() for t in batches[0]], warmup=3, stream=s)  # capture does not execute

        def sync_state():
            # start every compared step from identical state (in place: the
            # graph keeps its addresses)
            with torch.no_grad():
                for a, b in zip(m_eager.state_dict().values(), m_graph.state_dict().values()):
                    b.copy_(a)
                for pe, pg in zip(m_eager.parameters(), m_graph.parameters()):
                    o_g.state[pg]["momentum_buffer"].copy_(o_e.state[pe]["momentum_buffer"])

        def flat(ps):
            return torch.cat([p.detach().float().reshape(-1) for p in ps])

        for b in batches[1:5]:
            sync_state()
            torch.cuda.synchronize()
            p0 = flat(m_eager.parameters())
            le = run_e(*b).item()
            lg = cap(*b).item()
            torch.cuda.synchronize()
            assert abs(le - lg) < 1e-2 * max(1.0, abs(le)), (le, lg)
            # the whole update vector: per-parameter BN-bias grads of this tiny
            # random-init bf16 net differ by 10-30 % between two EAGER runs
            # (MIOpen / atomic-order noise, tools/graph_numerics.py); a stale or
            # missing captured input gives O(1) or non-finite differences
            de, dg = flat(m_eager.parameters()) - p0, flat(m_graph.parameters()) - p0
            assert bool(torch.isfinite(dg).all())
            rel = float((de - dg).norm() / de.norm().clamp_min(1e-12))
            assert rel < 0.3, rel
    finally:
        dcp.distributed.destroy_process_group()


def test_dropout_masks_fresh_per_replay(cuda):
    """The captured dropout reads the device Philox counter: each replay draws a
    new mask, and the captured backward regenerates the same mask."""
    from distributed_compute_pytorch_amd.ops import fused_dropout

    x = torch.randn(4096, device=cuda, requires_grad=True)
    fused_dropout(x, 0.5).sum().backward()  # eager warmup (creates the counter)
    x.grad = None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = fused_dropout(x, 0.5)
        y.sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    x.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        y = fused_dropout(x, 0.5)
        y.sum().backward()
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        m = y.detach() != 0
        assert torch.equal(x.grad != 0, m)
        masks.append(m.clone())
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])


def test_dropout_masks_fresh_per_replay_batched(cuda):
    """Inside ops.dropout.batched_offsets (what CapturedStep wraps a captured
    step in): the calls read the device counter itself and one add at the end
    advances it — every replay draws new masks, two calls of one replay draw
    different ones, and each backward regenerates its forward's mask."""
    from distributed_compute_pytorch_amd.ops import fused_dropout
    from distributed_compute_pytorch_amd.ops.dropout import batched_offsets

    x = torch.randn(4096, device=cuda, requires_grad=True)
    z = torch.randn(4096, device=cuda, requires_grad=True)
    (fused_dropout(x, 0.5).sum() + fused_dropout(z, 0.5).sum()).backward()  # eager warmup
    x.grad = z.grad = None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        (fused_dropout(x, 0.5).sum() + fused_dropout(z, 0.5).sum()).backward()
    torch.cuda.current_stream().wait_stream(s)
    x.grad = z.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        with batched_offsets():
            y = fused_dropout(x, 0.5)
            w = fused_dropout(z, 0.5)
            (y.sum() + w.sum()).backward()
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        m, n = y.detach() != 0, w.detach() != 0
        assert torch.equal(x.grad != 0, m) and torch.equal(z.grad != 0, n)
        assert not torch.equal(m, n)
        masks.append(m.clone())
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])


@pytest.mark.parametrize("gemm", [False, True])
def test_captured_fwd_bwd_matches_eager(cuda, gemm):
    """Forward + backward (+ our DDP) captured in one HIP graph: loss equal to
    eager, gradients within the eager-vs-eager noise of this bf16 net."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port
    from distributed_compute_pytorch_amd.models import resnet18_like
    from distributed_compute_pytorch_amd.utils.graphs import CapturedStep, capture_stream

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    try:
        torch.manual_seed(0)
        base = resnet18_like(num_classes=10, fused_bn=True, fused_gemm=gemm).to(cuda).to(
            memory_format=torch.channels_last)
        m_e, m_g = copy.deepcopy(base), copy.deepcopy(base)
        s = capture_stream()
        n_e = dcp.parallel.DistributedDataParallel(m_e, device_ids=[0], gradient_as_bucket_view=True)
        with torch.cuda.stream(s):
            n_g = dcp.parallel.DistributedDataParallel(m_g, device_ids=[0], gradient_as_bucket_view=True)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(8, 3, 64, 64, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (8,), generator=g).to(cuda)

        def make(net, model):
            def step(xx, yy):
                for p in model.parameters():
                    p.grad = None
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = F.cross_entropy(net(xx), yy)
                loss.backward()
                return loss
            return step

        st_e, st_g = make(n_e, m_e), make(n_g, m_g)
        for _ in range(3):
            st_e(x, y)
        cap = CapturedStep(st_g, [x.clone(), y.clone()], warmup=3, stream=s)
        with torch.no_grad():
            for a, b in zip(m_e.state_dict().values(), m_g.state_dict().values()):
                b.copy_(a)
        torch.cuda.synchronize()
        le = float(st_e(x, y).detach())
        ge = torch.cat([p.grad.detach().float().reshape(-1) for p in m_e.parameters()])
        with torch.no_grad():
            for a, b in zip(m_e.state_dict().values(), m_g.state_dict().values()):
                b.copy_(a)
        lg = float(cap(x, y).detach())
        torch.cuda.synchronize()
        gg = torch.cat([p.grad.detach().float().reshape(-1) for p in m_g.parameters()])
        le2 = float(st_e(x, y).detach())
        ge2 = torch.cat([p.grad.detach().float().reshape(-1) for p in m_e.parameters()])
        assert abs(le - lg) < 1e-2 * max(1.0, abs(le)), (le, lg, le2)
        noise = float((ge2 - ge).norm())
        err = float((gg - ge).norm())
        assert bool(torch.isfinite(gg).all())
        assert err < 3 * noise + 0.02 * float(ge.norm()), (err, noise, float(ge.norm()))
    finally:
        dcp.distributed.destroy_process_group()


@pytest.mark.parametrize("op", ["conv1x1", "conv_fwd", "bn_act_fwd", "colsum", "sgd_table"])
def test_captured_op_replays_equal_eager(cuda, op):
    """Every replay (not just the first) of a captured op equals eager: the
    zeroed accumulators and multi-tensor tables are built by kernels inside the
    graph, never by memset / memcpy nodes (which this ROCm does not order
    before the next kernel node on later replays)."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd._ext import C as _C

    torch.manual_seed(0)
    cl = torch.channels_last
    x = torch.randn(8, 64, 16, 16, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)
    w1 = torch.randn(64, 64, device=cuda).to(torch.bfloat16)
    w3 = torch.randn(64, 3, 3, 64, device=cuda).to(torch.bfloat16)
    g = torch.rand(64, device=cuda) + 0.5
    b = torch.randn(64, device=cuda)
    params = [torch.randn(n, device=cuda) for n in (3000, 17, 40000)]
    for p in params:
        p.grad = torch.randn_like(p)
    opt = dcp.optim.SGD(params, lr=0.1, momentum=0.9) if op == "sgd_table" else None
    fns = {
        "conv1x1": lambda: _C.conv1x1_fwd(x, w1, None, None, False, True),
        "conv_fwd": lambda: _C.conv_fwd(x, w3, 3, 3, 1, 1, True),
        "bn_act_fwd": lambda: _C.bn_act_fwd(x, g, b, None, None, None, True, 0.1, 1e-5, True, None, None)[:3],
        "colsum": lambda: [_C.colsum(x.permute(0, 2, 3, 1).reshape(-1, 64))],
    }
    if op == "sgd_table":
        opt.step()  # eager step creates the momentum buffers
        def fn():
            opt.step()
            return list(params)
    else:
        fn = fns[op]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s, capture_error_mode="thread_local"):
        out = fn()
    for i in range(3):
        if op == "sgd_table":
            # eager reference of one more step from the current state
            ref_p = [p.detach().clone() for p in params]
            ref_buf = [opt.state[p]["momentum_buffer"].clone() for p in params]
            for rp, rb, p in zip(ref_p, ref_buf, params):
                rb.mul_(0.9).add_(p.grad)
                rp.add_(rb, alpha=-0.1)
            gr.replay()
            torch.cuda.synchronize()
            for rp, p in zip(ref_p, params):
                torch.testing.assert_close(p, rp, rtol=1e-5, atol=1e-5)
        else:
            ref = [t.float().clone() for t in fn() if torch.is_tensor(t) and t.numel()]
            gr.replay()
            torch.cuda.synchronize()
            got = [t.float() for t in out if torch.is_tensor(t) and t.numel()]
            for a, r in zip(got, ref):
                torch.testing.assert_close(a, r, rtol=2e-3, atol=2e-3 * float(r.abs().max()) + 1e-6)


def test_captured_gpt2_step_matches_eager(cuda):
    """GPT-2 (fused linears / LN / attention / vocab xent, capture-safe embedding
    backward, capturable AdamW with device-side step counts): 4 replays of the
    captured step track 4 eager steps from the same start."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models.gpt2 import GPT2, GPT2Config
    from distributed_compute_pytorch_amd.utils.graphs import CapturedStep, capture_stream

    torch.manual_seed(0)
    cfg = GPT2Config(vocab_size=512, n_positions=128, n_embd=128, n_layer=2, n_head=2, dropout=0.0)
    base = GPT2(cfg).to(cuda)
    m_e, m_g = copy.deepcopy(base), copy.deepcopy(base)
    o_e = dcp.optim.AdamW(m_e.parameters(), lr=1e-3, weight_decay=0.1, capturable=True)
    s = capture_stream()
    with torch.cuda.stream(s):
        o_g = dcp.optim.AdamW(m_g.parameters(), lr=1e-3, weight_decay=0.1, capturable=True)
    g = torch.Generator().manual_seed(1)
    batches = []
    for _ in range(6):
        t = torch.randint(0, 512, (4, 129), generator=g)
        batches.append((t[:, :-1].contiguous().to(cuda), t[:, 1:].contiguous().to(cuda)))

    def make(m, opt):
        def run(x, y):
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(x, y)
            loss.backward()
            opt.step()
            return loss
        return run

    run_e, run_g = make(m_e, o_e), make(m_g, o_g)
    for _ in range(2):
        run_e(*batches[0])
    cap = CapturedStep(run_g, [t.clone() for t in batches[0]], warmup=2, stream=s)
    for b in batches[1:5]:
        le = float(run_e(*b).detach())
        lg = float(cap(*b).detach())
        assert abs(le - lg) < 2e-2 * max(1.0, abs(le)), (le, lg)
    pe = torch.cat([p.detach().float().reshape(-1) for p in m_e.parameters()])
    pg = torch.cat([p.detach().float().reshape(-1) for p in m_g.parameters()])
    assert bool(torch.isfinite(pg).all())
    assert float((pe - pg).norm() / pe.norm()) < 1e-2
