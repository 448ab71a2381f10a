"""hipBLASLt (torch.mm) vs our MFMA GEMMs on ResNet-50 b512 layer-3/4 1x1
shapes: fwd C[M,N] = A[M,K]·W[N,K]^T, wgrad D[N,K] = gy[M,N]^T·x[M,K].

    python tools/blas_vs_ours.py
"""
import json

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_compute_pytorch_amd._ext import C as _C


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = torch.device("cuda")
    for M, K, N in [(100352, 1024, 256), (100352, 256, 1024), (25088, 2048, 512), (25088, 512, 2048),
                    (401408, 512, 128), (401408, 128, 512)]:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        g = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fl = 2 * M * N * K
        x4 = a.view(M // 49, 7, 7, K).permute(0, 3, 1, 2)  # NHWC view as [n, K, 7, 7] channels_last
        g4 = g.view(M // 49, 7, 7, N).permute(0, 3, 1, 2)
        r = {"M": M, "K": K, "N": N}
        r["blas_fwd_us"] = bench(lambda: torch.mm(a, w.t()))
        r["ours_fwd_us"] = bench(lambda: _C.conv1x1_fwd(x4, w, None, None, False, False))
        r["ours_fwd_stats_us"] = bench(lambda: _C.conv1x1_fwd(x4, w, None, None, False, True))
        r["blas_wgrad_us"] = bench(lambda: torch.mm(g.t(), a))
        r["ours_wgrad_us"] = bench(lambda: _C.conv1x1_wgrad(g4, x4))
        for k in list(r):
            if k.endswith("_us"):
                r[k.replace("_us", "_TFps")] = round(fl / r[k] / 1e6, 1)
                r[k] = round(r[k], 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
