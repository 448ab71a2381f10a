"""In-process A/B of gemm_nt launcher variants (`_C.gemm_tune`) on every
ResNet-50 forward / data-gradient GEMM shape at one batch, against hipBLASLt
(torch.mm) on the plain shapes. Rounds are interleaved (variant order rotates
each round) and the median per variant is reported; outputs of every variant
are checked bit-equal to variant 0 first (the variants only change the
pipeline, not the per-element MFMA order).

    python tools/gemm_ab.py [--batch 512] [--rounds 5] [--iters 10] \
        [--variants nt_ns=0 nt_ns=3] [--json out.jsonl]
"""
import argparse
import json
import re
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def shapes(b):
    """(name, kind, H, Cin, Cout): kind 1x1 = stride-1 1x1 fwd(+stats) with a
    plain dgrad twin, 3x3 = stride-1 3x3 fwd(+stats) (also the dgrad shape)."""
    out = []
    for hw, ci, co in [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
                       (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048),
                       (7, 2048, 512)]:
        out.append((f"1x1 {hw}x{hw} {ci}->{co}", "1x1", hw, ci, co))
    for hw, c in [(28, 128), (14, 256), (7, 512)]:
        out.append((f"3x3 {hw}x{hw} {c}", "3x3", hw, c, c))
    return out


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", nargs="+", default=["nt_ns=0", "nt_ns=3"])
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bf, cl = torch.bfloat16, torch.channels_last
    variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in re.split("[,+]", v)) for v in a.variants]
    names = list(a.variants)

    def setv(v):
        for k, val in v.items():
            _C.gemm_tune(k, val)

    tot = {n: 0.0 for n in names + ["blas"]}
    out = open(a.json, "a") if a.json else None
    for name, kind, hw, ci, co in shapes(a.batch):
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(a.batch, ci, hw, hw, device=dev, generator=g) * 2 - 1).to(bf).contiguous(memory_format=cl)
        M = a.batch * hw * hw
        if kind == "1x1":
            w = ((torch.rand(co, ci, device=dev, generator=g) * 2 - 1) / ci ** 0.5).to(bf)
            gy = (torch.rand(a.batch, co, hw, hw, device=dev, generator=g) * 2 - 1).to(bf).contiguous(memory_format=cl)
            wt = w.t().contiguous()
            ops = {"fwd": lambda: _C.conv1x1_fwd(x, w, None, None, False, True),
                   "dgrad": lambda: _C.conv1x1_dgrad(gy, wt)}
            x2, gy2 = x.permute(0, 2, 3, 1).reshape(M, ci), gy.permute(0, 2, 3, 1).reshape(M, co)
            blas = {"fwd": lambda: torch.mm(x2, w.t()), "dgrad": lambda: torch.mm(gy2, w)}
            flops = 2.0 * M * ci * co
        else:
            w = ((torch.rand(co, 3, 3, ci, device=dev, generator=g) * 2 - 1) / (9 * ci) ** 0.5).to(bf).contiguous()
            ops = {"fwd": lambda: _C.conv_fwd(x, w, 3, 3, 1, 1, True)}
            blas = {}
            flops = 2.0 * M * ci * co * 9
        for op, fn in ops.items():
            ref = None
            for n, v in zip(names, variants):  # correctness: every variant bit-equal to the first
                setv(v)
                r = fn()
                r = r[0] if isinstance(r, (list, tuple)) else r
                torch.cuda.synchronize()
                if ref is None:
                    ref = r.clone()
                elif not torch.equal(ref, r):
                    d = (ref.float() - r.float()).abs().max().item()
                    print(json.dumps({"shape": name, "op": op, "variant": n, "MISMATCH_maxabs": d}), flush=True)
            times = {n: [] for n in names}
            bt = []
            for rd in range(a.rounds):
                order = list(range(len(names)))
                order = order[rd % len(order):] + order[:rd % len(order)]
                for i in order:
                    setv(variants[i])
                    fn()
                    torch.cuda.synchronize()
                    times[names[i]].append(timeit(fn, a.iters))
                if op in blas:
                    blas[op]()
                    torch.cuda.synchronize()
                    bt.append(timeit(blas[op], a.iters))
            row = {"shape": name, "op": op, "M": M}
            for n in names:
                us = statistics.median(times[n])
                row[n] = round(us, 1)
                row[n + "_TF"] = round(flops / us / 1e6, 1)
                tot[n] += us
            if bt:
                row["blas"] = round(statistics.median(bt), 1)
                row["blas_TF"] = round(flops / row["blas"] / 1e6, 1)
            print(json.dumps(row), flush=True)
            if out:
                out.write(json.dumps(row) + "\n")
    setv(variants[0])
    summ = {"total_us": {n: round(tot[n], 1) for n in names}}
    print(json.dumps(summ), flush=True)
    if out:
        out.write(json.dumps(summ) + "\n")


if __name__ == "__main__":
    main()
