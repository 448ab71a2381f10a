"""Full-size ResNet-50 on the production path (every default fusion: fused
stem, weight prep, BN-apply prologues, RED / RESRED epilogues, direct 3x3
kernels, residual-BN fusion; our DDP over RCCL) against the stock model in
fp32, at 224x224 with batch 32 — the kernels that make the headline number.

Reference: /root/reference/main.py:55-63 (one training step: forward, loss,
backward, optimizer) on the model family of BASELINE config #2.

Noise floor: the same stock model under bf16 autocast vs fp32 (same bf16-
rounded weights and inputs). Ours must be within 1.5x of that floor for every
parameter gradient, with no additive slack."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def pg(cuda):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    mine = not dcp.distributed.is_initialized()
    if mine:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
        dcp.distributed.init_process_group("rccl", device_id=0)
    yield dcp.distributed.get_default_group()
    if mine:
        dcp.distributed.destroy_process_group()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _models(cuda):
    from distributed_compute_pytorch_amd.models import resnet50

    torch.manual_seed(0)
    ref = resnet50(num_classes=1000).to(cuda).to(memory_format=CL)
    with torch.no_grad():  # bf16-rounded weights everywhere: weight rounding is not part of the error
        for p in ref.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    stock16 = resnet50(num_classes=1000).to(cuda).to(memory_format=CL)
    ours = resnet50(num_classes=1000, fused_bn=True).to(cuda).to(memory_format=CL)
    stock16.load_state_dict(ref.state_dict())
    ours.load_state_dict(ref.state_dict())
    return ref, stock16, ours


def _batch(cuda, g, n=32):
    x = torch.randn(n, 3, 224, 224, generator=g).to(torch.bfloat16).float()
    y = torch.randint(0, 1000, (n,), generator=g)
    return x.to(cuda).contiguous(memory_format=CL), y.to(cuda)


def test_resnet50_production_grads_within_bf16_noise(pg, cuda):
    import distributed_compute_pytorch_amd as dcp

    ref, stock16, ours = _models(cuda)
    ddp = dcp.parallel.DistributedDataParallel(ours, device_ids=[0], gradient_as_bucket_view=True,
                                               **dcp.parallel.XGMI_BUCKETS)
    g = torch.Generator().manual_seed(1)
    x, y = _batch(cuda, g)
    F.cross_entropy(ref(x), y).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        l16 = F.cross_entropy(stock16(x), y)
    l16.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lo = F.cross_entropy(ddp(x), y)
    lo.backward()
    torch.cuda.synchronize()
    rows, bad = [], []
    for (n, p32), p16, po in zip(ref.named_parameters(), stock16.parameters(), ours.parameters()):
        e16, eo = _rel(p16.grad, p32.grad), _rel(po.grad, p32.grad)
        rows.append((n, eo, e16))
        if not eo <= 1.5 * e16:
            bad.append((n, round(eo, 5), round(e16, 5)))
    worst = sorted(rows, key=lambda r: -r[1] / max(r[2], 1e-30))[:8]
    print("worst ours/stock-bf16 gradient error ratios:", [(n, round(a, 5), round(b, 5)) for n, a, b in worst])
    assert not bad, bad
    # running statistics (one training forward each): within 1e-2 of fp32, or
    # within 1.5x of stock bf16's own deviation where that is larger (deep
    # layers: the bf16 activations themselves differ from fp32 by ~1 %)
    for (n, b32), b16, bo in zip(ref.named_buffers(), stock16.buffers(), ours.buffers()):
        if b32.is_floating_point():
            assert _rel(bo, b32) < max(1e-2, 1.5 * _rel(b16, b32)), (n, _rel(bo, b32), _rel(b16, b32))
        else:
            assert torch.equal(bo, b32), n


def test_resnet50_production_loss_trajectory(pg, cuda):
    """16 SGD steps cycling over 4 fixed random 224x224 batches (a stable,
    memorising regime: the loss falls 7.07 -> ~5.05, so rounding differences
    are not amplified chaotically): ours (bf16, every fusion, our DDP + fused
    SGD) stays as close to the fp32 stock trajectory as the stock bf16 run
    does (≤ 2.5x its largest deviation so far, floor 1 % of the loss).
    Past step ~16 the fp32 loss itself stops falling and oscillates (5.05 ->
    5.20 -> 5.02 at steps 15 / 20 / 25): there every run's rounding is
    amplified, and a 30-step version failed on a late step in one of ~3 runs
    (round 6)."""
    import distributed_compute_pytorch_amd as dcp

    ref, stock16, ours = _models(cuda)
    ddp = dcp.parallel.DistributedDataParallel(ours, device_ids=[0], gradient_as_bucket_view=True,
                                               **dcp.parallel.XGMI_BUCKETS)
    lr = 0.005
    opts = [torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9),
            torch.optim.SGD(stock16.parameters(), lr=lr, momentum=0.9),
            dcp.optim.SGD(ddp.parameters(), lr=lr, momentum=0.9)]
    runs = [(ref, False), (stock16, True), (ddp, True)]
    losses = [[], [], []]
    g = torch.Generator().manual_seed(2)
    batches = [_batch(cuda, g) for _ in range(4)]
    for step in range(16):
        x, y = batches[step % 4]
        for k, ((m, amp), o) in enumerate(zip(runs, opts)):
            o.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            o.step()
            losses[k].append(loss.item())
    l32, l16, lo = (torch.tensor(v) for v in losses)
    print("loss fp32", l32[::5].tolist(), "bf16", l16[::5].tolist(), "ours", lo[::5].tolist())
    assert torch.isfinite(lo).all()
    assert l32[-4:].mean() < l32[:4].mean(), "the reference run is not in the stable regime the bound assumes"
    d16 = torch.maximum((l16 - l32).abs().cummax(0).values, 0.01 * l32.abs())
    do = (lo - l32).abs()
    # 2.5x: the runs are not bit-reproducible (atomic BN / wgrad reductions)
    assert (do <= 2.5 * d16).all(), (do.tolist(), d16.tolist())
