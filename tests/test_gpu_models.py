"""Transformer model families on the fused kernels vs the stock-op variants."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["gpt2", "bert"])
def test_fused_matches_stock_eval(cuda, name):
    from distributed_compute_pytorch_amd import models

    torch.manual_seed(0)
    if name == "gpt2":
        a = models.gpt2_small(n_layer=2, fused=True).to(cuda).eval()
        b = models.gpt2_small(n_layer=2, fused=False).to(cuda).eval()
        b.load_state_dict(a.state_dict())
        idx = torch.randint(0, 50257, (2, 128), device=cuda)
        args = (idx, idx.roll(-1, 1))
        kw = {}
    else:
        a = models.bert_base(layers=2, fused=True).to(cuda).eval()
        b = models.bert_base(layers=2, fused=False).to(cuda).eval()
        b.load_state_dict(a.state_dict())
        ids = torch.randint(0, 30522, (2, 128), device=cuda)
        pos = torch.randint(0, 128, (2, 20), device=cuda)
        args = (ids,)
        kw = dict(mlm_positions=pos, mlm_labels=torch.randint(0, 30522, (2, 20), device=cuda),
                  nsp_labels=torch.tensor([0, 1], device=cuda))
    for amp in (False, True):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            la = a(*args, **kw)
            lb = b(*args, **kw)
        torch.testing.assert_close(la.float(), lb.float(), rtol=2e-2 if amp else 1e-4, atol=2e-2 if amp else 1e-4)
        la.backward()
        lb.backward()
        for (n, p), q in zip(a.named_parameters(), b.parameters()):
            if p.grad is None:
                continue
            # (attention key biases have ~zero true gradient: floor the denominator)
            rel = (p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-3)
            assert rel < (0.1 if amp else 1e-3), (n, float(rel))
        a.zero_grad()
        b.zero_grad()


@pytest.mark.parametrize("name,kw", [("gpt2", dict(batch=2, seq_len=256, accum=2)),
                                     ("bert", dict(batch=4, seq_len=128)),
                                     ("resnet50", dict(batch=8)),
                                     ("convnet", dict(batch=32))])
def test_workload_steps_under_ddp(cuda, name, kw):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd import workloads
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    try:
        wl = workloads.build(name, cuda, **kw)
        ddp = dcp.parallel.DistributedDataParallel(wl.model, device_ids=[0], gradient_as_bucket_view=True)
        opt = wl.make_optimizer(ddp.parameters())
        step = workloads.make_step(wl, ddp, opt)
        losses = [float(step()) for _ in range(3)]
        assert all(torch.isfinite(torch.tensor(losses))), losses
    finally:
        dcp.distributed.destroy_process_group()


@pytest.mark.parametrize("amp", [False, True])
def test_gpt2_ddp_no_sync_accumulation_matches_local(cuda, amp):
    """GPT-2 (fused kernels) under our DDP with no_sync gradient accumulation
    over 2 micro-batches + fused AdamW, 2 optimizer steps, vs the same model
    trained locally with plain autograd accumulation (world_size 1: the
    all-reduce average is the identity, so any difference is the DDP /
    in-kernel accumulation path). fp32: parameter updates to 1e-4; bf16:
    updates against a noise floor of two local runs."""
    import copy

    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd import models
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    try:
        torch.manual_seed(0)
        base = models.gpt2_small(n_layer=2, dropout=0.0, fused=True).to(cuda)  # deterministic masks
        p0 = torch.cat([p.detach().float().reshape(-1) for p in base.parameters()])
        data = [torch.randint(0, 50257, (2, 129), device=cuda) for _ in range(4)]

        def train(use_ddp):
            m = copy.deepcopy(base)
            net = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True) \
                if use_ddp else m
            opt = dcp.optim.AdamW(net.parameters(), lr=1e-3, weight_decay=0.01)
            for s in range(2):
                opt.zero_grad(set_to_none=True)
                for k in range(2):
                    seq = data[2 * s + k]
                    ctx = net.no_sync() if (use_ddp and k == 0) else contextlib.nullcontext()
                    with ctx:
                        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                            loss = net(seq[:, :-1], seq[:, 1:]) / 2
                        loss.backward()
                opt.step()
            torch.cuda.synchronize()
            return torch.cat([p.detach().float().reshape(-1) for p in m.parameters()]) - p0

        import contextlib

        d_ddp, d_loc, d_loc2 = train(True), train(False), train(False)
        err = float((d_ddp - d_loc).norm() / d_loc.norm())
        if amp:
            noise = float((d_loc2 - d_loc).norm() / d_loc.norm())
            assert err < 4 * noise + 2e-2, (err, noise)
        else:
            assert err < 1e-4, err
    finally:
        dcp.distributed.destroy_process_group()
