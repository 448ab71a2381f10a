"""Eager vs HIP-graph-replayed gradients of one training step, per model
variant: locates which component makes a captured step differ numerically.

    python tools/graph_numerics.py
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29883")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import distributed_compute_pytorch_amd as dcp  # noqa: E402
from distributed_compute_pytorch_amd.models import resnet18_like  # noqa: E402
from distributed_compute_pytorch_amd.utils.graphs import CapturedStep, capture_stream  # noqa: E402

dev = torch.device("cuda", 0)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def run(name, ddp=True, **kw):
    torch.manual_seed(0)
    base = resnet18_like(num_classes=10, **kw).to(dev).to(memory_format=torch.channels_last)
    m_e, m_g = copy.deepcopy(base), copy.deepcopy(base)
    s = capture_stream()
    if ddp:
        n_e = dcp.parallel.DistributedDataParallel(m_e, device_ids=[0], gradient_as_bucket_view=True)
        with torch.cuda.stream(s):
            n_g = dcp.parallel.DistributedDataParallel(m_g, device_ids=[0], gradient_as_bucket_view=True)
    else:
        n_e, n_g = m_e, m_g
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g).to(dev)

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
    # identical state (running stats advanced by the warmups) before the compared step
    with torch.no_grad():
        for a, b in zip(m_e.state_dict().values(), m_g.state_dict().values()):
            b.copy_(a)
    torch.cuda.synchronize()
    le = float(st_e(x, y))
    ge = [p.grad.detach().clone() for p in m_e.parameters()]
    with torch.no_grad():
        for a, b in zip(m_e.state_dict().values(), m_g.state_dict().values()):
            b.copy_(a)
    # replay twice from the same state: run-to-run noise of the captured step itself
    lg = float(cap(x, y))
    gg = [p.grad.detach().clone() for p in m_g.parameters()]
    le2 = float(st_e(x, y))
    ge2 = [p.grad.detach().clone() for p in m_e.parameters()]
    worst = sorted(((rel(a, b), n) for (n, _), a, b in zip(m_e.named_parameters(), gg, ge)), reverse=True)[:4]
    noise = max(rel(a, b) for a, b in zip(ge2, ge))
    print(f"{name:34s} loss eager {le:.5f} graph {lg:.5f} | eager-vs-eager grad noise {noise:.2e} | "
          f"worst graph-vs-eager {[(round(r, 5), n) for r, n in worst]}", flush=True)


if __name__ == "__main__":
    dcp.distributed.init_process_group("rccl", device_id=0)
    run("stock ATen BN, no DDP", ddp=False, fused_bn=False)
    run("stock ATen BN + our DDP", fused_bn=False)
    run("fused BN, no dual, no gemm", fused_bn=True, dual_bn=False, fused_gemm=False)
    run("fused BN + dual, no gemm", fused_bn=True, fused_gemm=False)
    run("fused BN + dual + gemm", fused_bn=True, fused_gemm=True)
    dcp.distributed.destroy_process_group()
