"""Wave-quantisation probe of gemm_nt: TF/s of the plain 1x1 GEMM (+stats) at
row counts M whose 128x128 tile count is an exact multiple of the resident
workgroup slots (512) vs the ResNet-50 b512 row counts in between.

    python tools/gemm_quant.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    for K, N in [(1024, 256), (2048, 512), (512, 2048), (2304, 256)]:
        tn = N // 128
        for M in [128 * 512 // tn * r for r in (1, 2, 3, 4)] + [25088, 100352]:
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(bf)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(bf)
            us = timeit(lambda: _C.conv1x1_fwd(x, w, None, None, False, True))
            tiles = (M + 127) // 128 * tn
            print(json.dumps({"K": K, "N": N, "M": M, "tiles": tiles, "rounds": round(tiles / 512, 3),
                              "us": round(us, 1), "TF": round(2 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
