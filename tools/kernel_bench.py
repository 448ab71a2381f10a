"""Achieved HBM bandwidth of the hand-written kernels on the shapes the
workloads run (ResNet-50 b256 BN / max-pool, GPT-2 LayerNorm / cross-entropy
/ dropout, optimizer updates over a full model).

Bytes are the analytic minimum each op must move (every input read once,
every output written once); time is HIP-event time over `--iters` calls.
Run under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` for counter
evidence (gfx950 FETCH_SIZE reads half of a streaming read's bytes).

    python tools/kernel_bench.py [--iters 20] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd as dcp  # noqa: E402
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    res = []

    def rec(name, ms, nbytes):
        r = {"op": name, "us": round(ms * 1e3, 1), "GB": round(nbytes / 1e9, 3),
             "TB_per_s": round(nbytes / (ms * 1e-3) / 1e12, 2)}
        res.append(r)
        print(json.dumps(r), flush=True)

    cl = torch.channels_last
    for (n, c, h, w, resid) in [(256, 64, 56, 56, False), (256, 256, 56, 56, True), (256, 128, 28, 28, False),
                                (256, 1024, 14, 14, True), (256, 512, 7, 7, False)]:
        x = torch.randn(n, c, h, w, device=dev).to(bf).contiguous(memory_format=cl)
        r = torch.randn_like(x) if resid else None
        wgt, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        E = x.numel() * 2
        out = {}

        def fwd():
            out["o"] = _C.bn_act_fwd(x, wgt, b, rm, rv, r, True, 0.1, 1e-5, True)

        ms = timeit(fwd, a.iters)
        rec(f"bn_fwd{'+res' if resid else ''}+relu [{n},{c},{h},{w}] (stats + apply)", ms, E * (3 + (1 if resid else 0)))
        y, mean, invstd, bits = out["o"]
        gy = torch.randn_like(x)
        gy2 = torch.randn_like(x) if resid else None

        def bwd():
            _C.bn_act_bwd(gy, gy2, x, wgt, b, mean, invstd, y, True, resid, True, bits if resid else None)

        ms = timeit(bwd, a.iters)
        # reduce: gy (+gy2) + x (+bits) [+ write g]; apply: g + x → dx
        nb = E * (2 + (1 if resid else 0)) + (E // 16 if resid else 0) + (E if resid else 0) + E * 3
        rec(f"bn_bwd{'+res(dual)' if resid else ''}+relu [{n},{c},{h},{w}] (reduce + apply)", ms, nb)

    x = torch.randn(256, 64, 112, 112, device=dev).to(bf).contiguous(memory_format=cl)
    out = {}
    ms = timeit(lambda: out.__setitem__("o", _C.maxpool2d_fwd(x, 3, 2, 1)), a.iters)
    yo, idx = out["o"]
    rec("maxpool3x3s2 fwd [256,64,112,112]", ms, x.numel() * 2 + yo.numel() * 3)
    gy = torch.randn_like(yo)
    ms = timeit(lambda: _C.maxpool2d_bwd(gy, idx, list(x.shape), 3, 2, 1), a.iters)
    rec("maxpool3x3s2 bwd [256,64,112,112]", ms, gy.numel() * 3 + x.numel() * 2)

    T, D, V = 8 * 1024, 768, 50257
    xf = torch.randn(T, D, device=dev)
    lw, lb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    out = {}
    ms = timeit(lambda: out.__setitem__("o", _C.layer_norm_fwd(xf, lw, lb, 1e-5, bf)), a.iters)
    rec(f"layernorm fwd fp32->bf16 [{T},{D}]", ms, T * D * (4 + 2))
    yl, mu, rs = out["o"]
    dy = torch.randn(T, D, device=dev).to(bf)
    ms = timeit(lambda: _C.layer_norm_bwd(dy, xf, lw, lb, mu, rs), a.iters)
    rec(f"layernorm bwd [{T},{D}]", ms, T * D * (2 + 4 + 4))

    xb = torch.randn(2 * T, D, device=dev).to(bf)
    ms = timeit(lambda: out.__setitem__("o", _C.layer_norm_fwd(xb, lw, lb, 1e-5, bf)), a.iters)
    rec(f"layernorm fwd bf16 [{2 * T},{D}]", ms, 2 * T * D * (2 + 2))
    yl, mu, rs = out["o"]
    dyb = torch.randn(2 * T, D, device=dev).to(bf)
    ms = timeit(lambda: _C.layer_norm_bwd(dyb, xb, lw, lb, mu, rs), a.iters)
    rec(f"layernorm bwd bf16 [{2 * T},{D}]", ms, 2 * T * D * (2 + 2 + 2))

    logits = torch.randn(T, V, device=dev).to(bf)
    tgt = torch.randint(0, V, (T,), device=dev)
    out = {}
    ms = timeit(lambda: out.__setitem__("o", _C.cross_entropy_fwd(logits, tgt, -100, 0.0)), a.iters)
    rec(f"softmax-xent fwd [{T},{V}] bf16", ms, logits.numel() * 2)
    loss, lse = out["o"]
    dl = torch.full((1,), 1.0 / T, device=dev)
    ms = timeit(lambda: _C.cross_entropy_bwd(logits, tgt, lse, dl, -100, 0.0), a.iters)
    rec(f"softmax-xent bwd [{T},{V}] bf16", ms, logits.numel() * 4)

    xd = torch.randn(T * D * 4, device=dev).to(bf)
    rd = torch.randn_like(xd)
    ms = timeit(lambda: _C.dropout_fwd(xd, rd, 0.1, 1234, 0), a.iters)
    rec(f"dropout+residual [{T * D * 4}] bf16", ms, xd.numel() * 6)

    from distributed_compute_pytorch_amd.models import gpt2_small, resnet50

    for name, m, kind in [("resnet50", resnet50(), "sgd"), ("gpt2-small", gpt2_small(), "adamw")]:
        ps = [p.detach().to(dev) for p in m.parameters()]
        gs = [torch.randn_like(p) for p in ps]
        nel = sum(p.numel() for p in ps)
        if kind == "sgd":
            bufs = [torch.zeros_like(p) for p in ps]
            ms = timeit(lambda: _C.fused_sgd(ps, gs, bufs, 0.1, 0.9, 0.0, 1e-4, False, False, False, 1.0), a.iters)
            rec(f"fused SGD-momentum {name} ({nel / 1e6:.1f}M params, one launch)", ms, nel * 4 * 5)
        else:
            opt = dcp.optim.AdamW([torch.nn.Parameter(p) for p in ps], lr=1e-4)
            for p, g in zip(opt.param_groups[0]["params"], gs):
                p.grad = g
            ms = timeit(lambda: opt.step(), a.iters)
            rec(f"fused AdamW {name} ({nel / 1e6:.1f}M params, one launch)", ms, nel * 4 * 7)
        del m
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
