"""ResNet-50 1x1 forward GEMMs (BN-stats epilogue, the step's
gemm_nt<128,128,...,1,...> family) timed cold — a 1 GiB write evicts L2 and
the Infinity Cache before every call, as in the training step, where each
activation was written by other kernels long before it is read — and warm
(back-to-back calls, operands cache-resident). Our conv1x1_fwd (whatever
tile the launcher picks) vs the 256 x 256 ping-pong GEMM (no stats epilogue:
a bound) vs hipBLASLt. Median µs per call, one JSON line per shape.

    python tools/rn_gemm_cold.py [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402

SHAPES = [("l2 conv1 512->128", 512 * 28 * 28, 128, 512), ("l2 conv3 128->512", 512 * 28 * 28, 512, 128),
          ("l3 conv1 1024->256", 512 * 14 * 14, 256, 1024), ("l3 conv3 256->1024", 512 * 14 * 14, 1024, 256),
          ("l4 conv1 2048->512", 512 * 7 * 7, 512, 2048), ("l4 conv3 512->2048", 512 * 7 * 7, 2048, 512),
          ("l1 conv3 64->256", 512 * 56 * 56, 256, 64), ("l1 conv1 256->64", 512 * 56 * 56, 64, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    flush = torch.empty(1 << 28, device=dev)  # 1 GiB
    for name, M, N, K in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, device=dev, generator=g) - 0.5).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) - 0.5) / K ** 0.5).to(torch.bfloat16)
        def nt(f, v, deep=0):
            def run():
                C.gemm_tune("nt_a", v)
                C.gemm_tune("nt_deep", deep)
                return f()
            return run

        ops = {"ours_stats": nt(lambda: C.conv1x1_fwd(x, w, None, None, False, True), 0),
               "ours_stats_nt": nt(lambda: C.conv1x1_fwd(x, w, None, None, False, True), 1),
               "ours_stats_deep": nt(lambda: C.conv1x1_fwd(x, w, None, None, False, True), 0, 2),
               "ours": nt(lambda: C.conv1x1_fwd(x, w, None, None, False, False), 0),
               "blas": lambda: torch.mm(x, w.t())}
        if N % 8 == 0:
            ops["pp"] = lambda: C.gemm_pp(x, w)
        rec = {"shape": name, "M": M, "N": N, "K": K, "MB": round((M * K + M * N) * 2 / 1e6, 1)}
        for k, f in ops.items():
            f()
            cold, warm = [], []
            for _ in range(a.reps):
                flush.fill_(1.0)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                f()
                e.record()
                torch.cuda.synchronize()
                cold.append(s.elapsed_time(e) * 1e3)
            for _ in range(a.reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                f()
                e.record()
                torch.cuda.synchronize()
                warm.append(s.elapsed_time(e) * 1e3)
            rec[k + "_cold_us"] = round(statistics.median(cold), 1)
            rec[k + "_warm_us"] = round(statistics.median(warm), 1)
        C.gemm_tune("nt_deep", 0)
        rec["cold_TBps_ours_stats"] = round(rec["MB"] / rec["ours_stats_cold_us"], 2)
        print(json.dumps(rec), flush=True)
        del x, w


if __name__ == "__main__":
    main()
