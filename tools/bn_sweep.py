"""BatchNorm kernels on every ResNet-50 b256 BN shape, split into the pieces the
GEMM path runs: statistics only (``bn_stats_coef``), apply with precomputed
statistics (``bn_act_fwd(stats=…)``), backward reduce + apply
(``bn_act_bwd``). One JSON line per shape with µs and achieved TB/s (analytic
minimum bytes). Geometry knobs are env vars read by the extension
(``DCP_BN_RED_BLOCKS``, ``DCP_BN_RED_ATOMICS``), so sweep them across processes.

    DCP_BN_RED_BLOCKS=1024 python tools/bn_sweep.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402

# (C, H=W, residual, calls per ResNet-50 step)
SHAPES = [(64, 56, False, 6), (128, 56, False, 1), (128, 28, False, 7), (256, 28, False, 1), (256, 14, False, 11),
          (512, 14, False, 1), (512, 7, False, 5), (256, 56, True, 3), (512, 28, True, 4), (1024, 14, True, 6),
          (2048, 7, True, 3)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    tot = {"stats": 0.0, "apply": 0.0, "bwd": 0.0, "ideal": 0.0}
    tag = {k: v for k, v in os.environ.items() if k.startswith("DCP_BN")}
    for c, hw, resid, calls in SHAPES:
        x = torch.randn(a.batch, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
        r = torch.randn_like(x) if resid else None
        w, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        E = x.numel() * 2
        us_s = timeit(lambda: _C.bn_stats_coef(x, w, b, rm, rv, 0.1, 1e-5, None), a.iters)
        sums = torch.stack([x.float().sum((0, 2, 3)), x.float().pow(2).sum((0, 2, 3))]).reshape(-1).contiguous()
        out = {}
        us_a = timeit(lambda: out.__setitem__("o", _C.bn_act_fwd(x, w, b, rm, rv, r, True, 0.1, 1e-5, True, None,
                                                                 sums)), a.iters)
        y, mean, invstd, bits = out["o"]
        gy = torch.randn_like(x)
        gy2 = torch.randn_like(x) if resid else None
        us_b = timeit(lambda: _C.bn_act_bwd(gy, gy2, x, w, b, mean, invstd, y, True, resid, True,
                                            bits if resid else None), a.iters)
        nb_s = E
        nb_a = E * (2 + (1 if resid else 0))
        nb_b = E * (2 + (1 if resid else 0)) + (E // 16 if resid else 0) + (E if resid else 0) + E * 3
        row = {"C": c, "HW": hw, "res": resid, "stats_us": round(us_s, 1), "stats_TBps": round(nb_s / us_s / 1e6, 2),
               "apply_us": round(us_a, 1), "apply_TBps": round(nb_a / us_a / 1e6, 2), "bwd_us": round(us_b, 1),
               "bwd_TBps": round(nb_b / us_b / 1e6, 2)}
        print(json.dumps(row), flush=True)
        tot["stats"] += us_s * calls
        tot["apply"] += us_a * calls
        tot["bwd"] += us_b * calls
        tot["ideal"] += (nb_s + nb_a + nb_b) / 5e6 * calls  # at 5 TB/s
    print(json.dumps({"env": tag, "weighted_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
