"""Eager vs HIP-graph replay numerics of a whole training step, by variant.

Two copies of one model take the same warmup steps (eager / on the capture
stream); the graph copy is then captured once and both run the same next
batches. Losses and parameter drift are printed per variant so a broken
component (fused BN, DDP, our optimizer) shows up as the first diverging row.

    python tools/graph_opt_debug.py
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29882")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import distributed_compute_pytorch_amd as dcp  # noqa: E402
from distributed_compute_pytorch_amd.models import resnet18_like  # noqa: E402

dev = torch.device("cuda", 0)
dcp.distributed.init_process_group("rccl", device_id=0)


def run(name, fused, gemm, use_ddp, opt_kind, fwd_only_loss=False):
    torch.manual_seed(0)
    base = resnet18_like(num_classes=10, fused_bn=fused, fused_gemm=gemm).to(dev).to(memory_format=torch.channels_last)
    g = torch.Generator().manual_seed(1)
    batches = [(torch.randn(8, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last),
                torch.randint(0, 10, (8,), generator=g).to(dev)) for _ in range(6)]
    s = torch.cuda.Stream()
    nets = []
    for which in ("eager", "graph"):
        m = copy.deepcopy(base)
        ctx = torch.cuda.stream(s) if which == "graph" else torch.cuda.stream(torch.cuda.current_stream())
        with ctx:
            net = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True) \
                if use_ddp else m
            if opt_kind == "ours":
                opt = dcp.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
            else:
                opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
        nets.append((m, net, opt))

    def make(net, opt, static=None):
        def step(x, y):
            if opt is not None:
                opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(net(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    (me, ne, oe), (mg, ng, og) = nets
    se, sg = make(ne, oe), make(ng, og)
    for b in batches[:3]:
        se(*b)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for b in batches[:3]:
            sg(*b)
    torch.cuda.synchronize()
    static = [t.clone() for t in batches[3]]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
        out = sg(*static)
    torch.cuda.synchronize()

    def flat(m):
        return torch.cat([p.detach().float().reshape(-1) for p in m.parameters()])

    rows = []
    for b in batches[3:]:
        le = float(se(*b))
        for d, src in zip(static, b):
            d.copy_(src)
        graph.replay()
        torch.cuda.synchronize()
        lg = float(out)
        pe, pg = flat(me), flat(mg)
        rows.append((le, lg, float((pe - pg).norm() / pe.norm())))
    print(f"{name:45s} " + "  ".join(f"eager {a:.4f} graph {b:.4g} pdrift {c:.2e}" for a, b, c in rows), flush=True)


for fused, gemm in ((False, False), (True, False), (True, True)):
    for use_ddp in (False, True):
        for opt_kind in ("torch", "ours"):
            try:
                run(f"fused={fused} gemm={gemm} ddp={use_ddp} opt={opt_kind}", fused, gemm, use_ddp, opt_kind)
            except Exception as e:  # noqa: BLE001
                print(f"fused={fused} gemm={gemm} ddp={use_ddp} opt={opt_kind}: {type(e).__name__}: "
                      f"{str(e).splitlines()[0][:200]}", flush=True)
                torch.cuda.synchronize()
