"""One 1x1-conv GEMM shape, repeated (a small target for rocprofv3 --pmc).

    python tools/gemm_one.py --m 12544 --cin 2048 --cout 512 --op fwd [--iters 10]
op: fwd | fwd_pro | dgrad | wgrad | conv3 (3x3 stride-1 implicit GEMM fwd, --hw spatial) | wgrad3 (its weight gradient)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=12544)
    ap.add_argument("--cin", type=int, default=2048)
    ap.add_argument("--cout", type=int, default=512)
    ap.add_argument("--op", default="fwd")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--hw", type=int, default=14)
    ap.add_argument("--tune", nargs="*", default=[], help="gemm_tune key=value pairs (e.g. nt_big=2)")
    a = ap.parse_args()
    for kv in a.tune:
        k, v = kv.split("=")
        _C.gemm_tune(k, int(v))
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    x = (torch.rand(1, a.cin, a.m, 1, device=dev) * 2 - 1).to(bf).contiguous(memory_format=torch.channels_last)
    gy = (torch.rand(1, a.cout, a.m, 1, device=dev) * 2 - 1).to(bf).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(a.cout, a.cin, device=dev) / a.cin ** 0.5).to(bf)
    wt = w.t().contiguous()
    sc, sf = torch.ones(a.cin, device=dev), torch.zeros(a.cin, device=dev)
    if a.op == "wgrad3":
        n = a.m // (a.hw * a.hw)
        xi = torch.randn(n, a.cin, a.hw, a.hw, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
        gi = torch.randn(n, a.cout, a.hw, a.hw, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
        for _ in range(a.iters):
            _C.conv_wgrad(gi, xi, 3, 3, 1, 1)
        torch.cuda.synchronize()
        print("ok", flush=True)
        return
    if a.op == "conv3":
        n = a.m // (a.hw * a.hw)
        xi = torch.randn(n, a.cin, a.hw, a.hw, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
        w3 = (torch.randn(a.cout, 3, 3, a.cin, device=dev) / (9 * a.cin) ** 0.5).to(bf).contiguous()
        for _ in range(a.iters):
            _C.conv_fwd(xi, w3, 3, 3, 1, 1, True)
        torch.cuda.synchronize()
        print("ok", flush=True)
        return
    fn = {"fwd": lambda: _C.conv1x1_fwd(x, w, None, None, False, False),
          "fwd_pro": lambda: _C.conv1x1_fwd(x, w, sc, sf, True, False),
          "dgrad": lambda: _C.conv1x1_dgrad(gy, wt),
          "wgrad": lambda: _C.conv1x1_wgrad(gy, x)}[a.op]
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
