"""Which component turns HIP-graph replays non-finite?

Eager and graph copies of one model take the same warmup steps, the graph copy
is captured once, then both run the same batches; after every replay the
parameters / grads / buffers of the graph copy that are non-finite are listed
by name, so the first broken op shows up. Variants toggle the fused stem, the
weight prep, autocast's weight cache and the model family (a stock-torch net is
the control: if it breaks, capture itself is the problem).

    python tools/graph_nan_debug.py
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_compute_pytorch_amd.models.resnet as R  # noqa: E402

dev = torch.device("cuda", 0)


def stock_net():
    return nn.Sequential(nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(),
                         nn.Conv2d(32, 64, 3, 2, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                         nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(64, 10))


def bad(m):
    out = []
    for n, p in m.named_parameters():
        if not bool(torch.isfinite(p).all()):
            out.append("P:" + n)
        if p.grad is not None and not bool(torch.isfinite(p.grad).all()):
            out.append("G:" + n)
    for n, b in m.named_buffers():
        if b.is_floating_point() and not bool(torch.isfinite(b).all()):
            out.append("B:" + n)
    return out


def run(name, make_model, stem=True, prep=True, cache=True, lr=0.01):
    R.FUSED_STEM, R.WEIGHT_PREP = stem, prep
    torch.manual_seed(0)
    base = make_model().to(dev).to(memory_format=torch.channels_last)
    g = torch.Generator().manual_seed(1)
    batches = [(torch.randn(8, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last),
                torch.randint(0, 10, (8,), generator=g).to(dev)) for _ in range(7)]
    s = torch.cuda.Stream()
    me, mg = copy.deepcopy(base), copy.deepcopy(base)
    oe = torch.optim.SGD(me.parameters(), lr=lr, momentum=0.9)
    og = torch.optim.SGD(mg.parameters(), lr=lr, momentum=0.9)

    def make(m, opt):
        def step(x, y):
            opt.zero_grad(set_to_none=False)
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=cache):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss.detach()
        return step

    se, sg = make(me, oe), make(mg, og)
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
    rows = []
    for i, b in enumerate(batches[3:]):
        le = float(se(*b))
        for d, src in zip(static, b):
            d.copy_(src)
        graph.replay()
        torch.cuda.synchronize()
        lg = float(out)
        bb = bad(mg)
        pe = torch.cat([p.detach().float().reshape(-1) for p in me.parameters()])
        pg = torch.cat([p.detach().float().reshape(-1) for p in mg.parameters()])
        rows.append(f"[{i}] e {le:.4f} g {lg:.4g} drift {float((pe - pg).norm() / pe.norm()):.2e}"
                    + (f" BAD {len(bb)}: {bb[:3]} .. {bb[-3:]}" if bb else ""))
        if bb:
            break
    print(f"{name:32s} " + " | ".join(rows), flush=True)


variants = [
    ("stock", stock_net, {}),
    ("stock nocache", stock_net, {"cache": False}),
    ("r18 plain nostem", lambda: R.resnet18_like(num_classes=10, fused_bn=False, fused_gemm=False), {"stem": False}),
    ("r18 plain nostem nocache", lambda: R.resnet18_like(num_classes=10, fused_bn=False, fused_gemm=False),
     {"stem": False, "cache": False}),
    ("r18 plain stem", lambda: R.resnet18_like(num_classes=10, fused_bn=False, fused_gemm=False), {}),
    ("r18 bn nostem", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=False), {"stem": False}),
    ("r18 gemm nostem noprep", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=True),
     {"stem": False, "prep": False}),
    ("r18 gemm nostem prep", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=True),
     {"stem": False}),
    ("r18 gemm all", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=True), {}),
    ("r18 gemm all lr1e-3", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=True), {"lr": 1e-3}),
]
only = sys.argv[1:]
for name, mk, kw in variants:
    if only and not any(o in name for o in only):
        continue
    try:
        run(name, mk, **kw)
    except Exception as e:  # noqa: BLE001
        print(f"{name:32s} {type(e).__name__}: {str(e).splitlines()[0][:200]}", flush=True)
        torch.cuda.synchronize()
