"""Single-GPU DDP path over RCCL (world_size 1): reducer, buckets, hooks."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(cuda):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    yield dcp.distributed.get_default_group()
    dcp.distributed.destroy_process_group()


def test_rccl_collectives(pg, cuda):
    import distributed_compute_pytorch_amd as dcp

    t = torch.arange(10, dtype=torch.float32, device=cuda)
    dcp.distributed.all_reduce(t)
    torch.testing.assert_close(t, torch.arange(10, dtype=torch.float32, device=cuda))
    out = torch.empty(10, device=cuda)
    dcp.distributed.all_gather_into_tensor(out, t)
    torch.testing.assert_close(out, t)
    dcp.distributed.broadcast(t, 0)
    dcp.distributed.barrier()
    assert pg.rccl_comm().backend == "rccl"


@pytest.mark.parametrize("grad_as_view", [False, True])
def test_ddp_matches_local_training(pg, cuda, grad_as_view):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet

    torch.manual_seed(0)
    ref = ConvNet().to(cuda)
    ours = ConvNet().to(cuda)
    ours.load_state_dict(ref.state_dict())
    ddp = dcp.parallel.DistributedDataParallel(ours, device_ids=[0], gradient_as_bucket_view=grad_as_view,
                                               bucket_cap_mb=1)
    o1 = torch.optim.Adadelta(ref.parameters(), lr=1e-3)
    o2 = dcp.optim.Adadelta(ddp.parameters(), lr=1e-3)
    ref.eval(), ours.eval()  # no dropout: deterministic comparison
    for it in range(3):
        x = torch.randn(16, 1, 28, 28, device=cuda)
        y = torch.randint(0, 10, (16,), device=cuda)
        for m, o in ((ref, o1), (ddp, o2)):
            o.zero_grad()
            with torch.enable_grad():
                F.nll_loss(m(x), y).backward()
            o.step()
    for p, q in zip(ref.parameters(), ours.parameters()):
        torch.testing.assert_close(q, p, rtol=1e-4, atol=1e-5)
    assert set(ddp.state_dict().keys()) == {"module." + k for k in ref.state_dict().keys()}


def test_resnet_grads_match_fp64_reference(pg, cuda):
    """One fp32 step: every parameter gradient through our DDP + fused BN
    against a deterministic fp64 CPU oracle of the same model, input and
    labels, with the reduced-precision fp32 paths pinned off
    (``allow_tf32 = False``).

    Bounds (no additive slack): the median parameter within 1.25x of the
    error fp32 arithmetic itself reaches on the CPU, and every parameter
    within 5x of the worse of two fp32 references — the CPU run and stock
    PyTorch (MIOpen convolutions + BatchNorm) on this GPU, the latter's error
    taken as the largest of three runs: its run-to-run spread on the
    ill-conditioned last-block BN gradients is ~5x (layer4.2.bn3.weight at
    5.0e-4 in one run, 2.3e-3 in another), and one run that lands low failed
    ours at 3.5e-3 (round-6 GPU run).
    Why not a flat multiple of the CPU error (NOTES §31,
    tools/resnet_fp64_diag.py, profiles/r6_fp64_diag_tf32*.txt): a
    random-init ResNet-50's last-block BN gradients are sums with heavy
    cancellation, so each fp32 run's forward rounding (1e-7 at the stem,
    ~8e-5 at layer 4 — ours within 1.2x of stock's) is amplified 10-100x and
    differently for every summation order: stock fp32 on this GPU is itself
    2-4x the CPU's error there, and the run-to-run spread of both GPU runs
    (atomic BN / MIOpen reductions) is ~2x. TF32 on or off moves none of it."""
    import copy

    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import resnet50

    tf32 = torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32
    torch.backends.cudnn.allow_tf32 = torch.backends.cuda.matmul.allow_tf32 = False
    try:
        torch.manual_seed(0)
        cpu = resnet50(num_classes=100)
        g = torch.Generator(device="cpu").manual_seed(0)
        x = torch.randn(16, 3, 96, 96, generator=g)
        y = torch.randint(0, 100, (16,), generator=g)
        ref64 = copy.deepcopy(cpu).double()
        l64 = F.cross_entropy(ref64(x.double()), y)
        l64.backward()
        ref32 = copy.deepcopy(cpu)
        F.cross_entropy(ref32(x), y).backward()
        xc, yc = x.to(cuda).contiguous(memory_format=torch.channels_last), y.to(cuda)
        stocks = []
        for _ in range(3):
            stock = copy.deepcopy(cpu).to(cuda).to(memory_format=torch.channels_last)
            F.cross_entropy(stock(xc), yc).backward()
            stocks.append(stock)
        model = resnet50(num_classes=100, fused_bn=True)
        model.load_state_dict(cpu.state_dict())
        model = model.to(cuda).to(memory_format=torch.channels_last)
        ddp = dcp.parallel.DistributedDataParallel(model, device_ids=[0], gradient_as_bucket_view=True)
        l2 = F.cross_entropy(ddp(xc), yc)
        l2.backward()
    finally:
        torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32 = tf32
    assert abs(float(l2) - float(l64)) < 1e-4 * abs(float(l64))
    ratios = []
    for (n, p64), p32, pss, q in zip(ref64.named_parameters(), ref32.parameters(),
                                     zip(*(st.parameters() for st in stocks)), model.parameters()):
        den = p64.grad.norm().clamp_min(1e-30)
        e32 = float((p32.grad.double() - p64.grad).norm() / den)
        est = max(float((ps.grad.double().cpu() - p64.grad).norm() / den) for ps in pss)
        ours = float((q.grad.double().cpu() - p64.grad).norm() / den)
        ratios.append(ours / max(e32, 1e-12))
        assert ours <= 5 * max(e32, est) or ours < 1e-6, (n, ours, e32, est)
    ratios.sort()
    assert ratios[len(ratios) // 2] <= 1.25, ratios[len(ratios) // 2]  # typically as accurate as fp32 on the CPU
    for (n, b64), c in zip(ref64.named_buffers(), model.buffers()):
        torch.testing.assert_close(c.double().cpu(), b64.double(), rtol=1e-4, atol=1e-5, msg=n)


def test_resnet_bf16_loss_tracks_stock(pg, cuda):
    """bf16 autocast, 3 SGD steps: loss trajectories agree within bf16 noise."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import resnet50

    torch.manual_seed(0)
    ref = resnet50(num_classes=100).to(cuda).to(memory_format=torch.channels_last)
    model = resnet50(num_classes=100, fused_bn=True).to(cuda).to(memory_format=torch.channels_last)
    model.load_state_dict(ref.state_dict())
    ddp = dcp.parallel.DistributedDataParallel(model, device_ids=[0], gradient_as_bucket_view=True)
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9)
    opt = dcp.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(16, 3, 128, 128, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (16,), generator=g).to(cuda)
    l_ref, l_ours = [], []
    for _ in range(3):
        for m, o, acc in ((ref, o_ref, l_ref), (ddp, opt, l_ours)):
            o.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            o.step()
            acc.append(loss.item())
    assert all(torch.isfinite(torch.tensor(l_ours)))
    assert l_ours[-1] < l_ours[0]
    for a, b in zip(l_ref, l_ours):
        assert abs(a - b) < 0.08 * max(1.0, abs(a)), (l_ref, l_ours)
    info = ddp.ddp_logging_data()
    assert info["rebuilds"] == 1 and sum(info["bucket_sizes"]) == sum(p.numel() * 4 for p in model.parameters())
