"""Replay-to-replay consistency of a captured training step.

With the optimizer step left out (or lr = 0) and the same input every replay,
every replay must produce the same loss and gradients as the eager step: a
drift from replay to replay means captured state that is not re-initialised
inside the graph (an accumulator zeroed only outside the capture, a buffer
swapped at capture time, ...). Variants isolate the fused components.

    python tools/graph_replay_check.py [name-filter ...]
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_compute_pytorch_amd.models.resnet as R  # noqa: E402
from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d  # noqa: E402
from distributed_compute_pytorch_amd.ops.pool import FusedMaxPool2d  # noqa: E402

dev = torch.device("cuda", 0)


class BNNet(nn.Module):
    def __init__(self, dual=False, residual=False, pool=False):
        super().__init__()
        self.c1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.b1 = BatchNormAct2d(64, act=True, fused=True)
        self.pool = FusedMaxPool2d(3, 2, 1) if pool else None
        self.c2 = nn.Conv2d(64, 64, 3, 1, 1, bias=False)
        self.b2 = BatchNormAct2d(64, act=True, residual=residual, fused=True)
        self.dual, self.residual = dual, residual
        self.fc = nn.Linear(64, 10)

    def forward(self, x):
        if self.dual:
            y, a = self.b1(self.c1(x), dual=True)
        else:
            y = self.b1(self.c1(x))
            a = y
        if self.pool is not None:
            y, a = self.pool(y, dual=True) if self.dual else (self.pool(y),) * 2
        z = self.b2(self.c2(y), a if self.residual else None)
        return self.fc(z.mean((2, 3)))


class GemmNet(nn.Module):
    """Only our kernels (no MIOpen): 3x3 implicit-GEMM conv, fused BN, 1x1 GEMM
    conv, fused BN(+residual); 64-channel bf16 input."""

    def __init__(self, residual=False):
        super().__init__()
        self.c1 = nn.Conv2d(64, 64, 3, 1, 1, bias=False)
        self.b1 = BatchNormAct2d(64, act=True, fused=True)
        self.c2 = nn.Conv2d(64, 64, 1, bias=False)
        self.b2 = BatchNormAct2d(64, act=True, residual=residual, fused=True)
        self.residual = residual
        self.fc = nn.Linear(64, 10)

    def forward(self, x):
        from distributed_compute_pytorch_amd.ops.conv import conv1x1, conv_kxk_gemm
        x = x.to(torch.bfloat16)
        z1, s1 = conv_kxk_gemm(x, self.c1.weight, 1, 1, stats=True)
        y1 = self.b1(z1, stats=s1)
        z2, s2 = conv1x1(y1, self.c2.weight, stats=True)
        z = self.b2(z2, y1 if self.residual else None, stats=s2)
        return self.fc(z.float().mean((2, 3)))


def run(name, make, opt_kind=None, steps=4, lr=0.0, mode="eager+sync"):
    torch.manual_seed(0)
    base = make().to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(8, 64 if isinstance(base, GemmNet) else 3, 32, 32, device=dev).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    s = torch.cuda.Stream()
    nets = []
    for which in ("eager", "graph"):
        m = copy.deepcopy(base)
        opt = None
        if opt_kind == "torch":
            opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9)
        elif opt_kind == "ours":
            import distributed_compute_pytorch_amd as dcp
            opt = dcp.optim.SGD(m.parameters(), lr=lr, momentum=0.9)
        nets.append((m, opt))

    def make_step(m, opt):
        def step():
            if opt is not None:
                opt.zero_grad(set_to_none=False)
            else:
                for p in m.parameters():
                    p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            if opt is not None:
                opt.step()
            return loss.detach()
        return step

    (me, oe), (mg, og) = nets
    se, sg = make_step(me, oe), make_step(mg, og)
    for _ in range(3):
        se()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            sg()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        from distributed_compute_pytorch_amd._ext import C as _C
        st_cur = _C.stream_capture_status(torch.cuda.current_stream().cuda_stream)
        out = sg()
    torch.cuda.synchronize()
    name = f"{name} cap={st_cur}"

    def sync():  # graph copy <- eager copy, in place (the graph keeps its addresses)
        with torch.no_grad():
            for a, b in zip(me.state_dict().values(), mg.state_dict().values()):
                b.copy_(a)
            if oe is not None:
                for pe, pg in zip(me.parameters(), mg.parameters()):
                    for k, v in oe.state[pe].items():
                        if torch.is_tensor(v):
                            og.state[pg][k].copy_(v)

    rows = []
    if "sync" in mode:
        sync()
    for i in range(steps):
        if i == 2 and "sync" in mode:
            sync()  # replay from the eager state once more: isolates per-step error from drift
        if "eager" in mode:
            le = float(se())
        else:
            le = float("nan")
        if "junk" in mode:  # unrelated allocations + writes between replays
            junk = [torch.full((1 << 20,), 7.0, device=dev) for _ in range(64)]
            del junk
        g.replay()
        torch.cuda.synchronize()
        lg = float(out)
        worst = sorted(((float((pg.detach() - pe.detach()).float().norm() / pe.detach().float().norm().clamp_min(1e-12)), n)
                        for (n, pe), pg in zip(me.named_parameters(), mg.parameters())), reverse=True)[:2]
        rows.append(f"{le:.4f}/{lg:.4g} [{', '.join(f'{n}={v:.1e}' for v, n in worst)}]")
    print(f"{name:28s} {mode:12s} lr={lr}: " + " | ".join(rows), flush=True)


variants = [
    ("gemm", lambda: GemmNet()),
    ("gemm res", lambda: GemmNet(residual=True)),
    ("bn", lambda: BNNet()),
    ("bn dual", lambda: BNNet(dual=True)),
    ("bn res", lambda: BNNet(residual=True)),
    ("bn dual res", lambda: BNNet(dual=True, residual=True)),
    ("bn pool", lambda: BNNet(pool=True)),
    ("bn dual pool res", lambda: BNNet(dual=True, pool=True, residual=True)),
    ("r18 bn nostem", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=False)),
    ("r18 gemm", lambda: R.resnet18_like(num_classes=10, fused_bn=True, fused_gemm=True)),
]
only = sys.argv[1:]
for name, mk in variants:
    if only and not any(o == name for o in only):
        continue
    for ok, lr, mode in (("torch", 0.0, "eager+sync"), ("torch", 0.0, "eager"), ("torch", 0.0, "sync"),
                         ("torch", 0.0, "junk"), ("torch", 0.0, "none")):
        try:
            run(f"{name} opt={ok}", mk, ok, lr=lr, mode=mode)
        except Exception as e:  # noqa: BLE001
            print(f"{name} opt={ok}: {type(e).__name__}: {str(e).splitlines()[0][:200]}", flush=True)
            torch.cuda.synchronize()
