"""BN-prologue 1x1 GEMM at the ResNet-50 conv3 shapes (BN2 + ReLU applied to
the A operand): plain GEMM (+ stats), the prologue on the BK = 32 ring
(pro_pipe 0) and on the pipelined BK = 64 loop (pro_pipe 1), and the separate
BN-apply pass the prologue replaces. One JSON line per shape (µs, best of 5 x 10)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402

dev = torch.device("cuda", 0)
bf = torch.bfloat16
SHAPES = [(512, 56, 64, 256), (512, 28, 128, 512), (512, 14, 256, 1024), (512, 7, 512, 2048)]


def t_us(fn, iters=10, reps=5):
    best = 1e30
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / iters)
    return round(best, 1)


for n, hw, ci, co in SHAPES:
    x = torch.randn(n, ci, hw, hw, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, ci, device=dev) / ci ** 0.5).to(bf)
    sc = torch.rand(ci, device=dev) + 0.5
    sf = torch.randn(ci, device=dev)
    g, b = torch.ones(ci, device=dev), torch.zeros(ci, device=dev)
    rm, rv = torch.zeros(ci, device=dev), torch.ones(ci, device=dev)
    xf = x.float().permute(0, 2, 3, 1).reshape(-1, ci)
    sums = torch.cat([xf.sum(0), (xf * xf).sum(0)])
    del xf
    r = {"shape": [n, hw, hw, ci, co]}
    r["plain_stats"] = t_us(lambda: C.conv1x1_fwd(x, w, None, None, False, True))
    r["apply_pass"] = t_us(lambda: C.bn_act_fwd(x, g, b, rm, rv, None, True, 0.1, 1e-5, True, None, sums))
    for pp in (0, 1):
        C.gemm_tune("pro_pipe", pp)
        r[f"pro_pipe{pp}"] = t_us(lambda: C.conv1x1_fwd(x, w, sc, sf, True, True))
    C.gemm_tune("pro_pipe", 0)
    r["unfused"] = round(r["plain_stats"] + r["apply_pass"], 1)
    print(json.dumps(r), flush=True)
