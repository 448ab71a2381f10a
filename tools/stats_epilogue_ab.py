"""ResNet-50 1x1 forward GEMMs with and without the BN-statistics epilogue
(VERDICT r4 Next 5): conv1x1_fwd(x, w, stats=False / True) at the bench's
batch-512 shapes, interleaved rounds, median µs and the compulsory-traffic
rate (read x + w, write y).

    python tools/stats_epilogue_ab.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402

SHAPES = [  # (name, N, H, W, Cin, Cout)
    ("l1_conv1", 512, 56, 56, 256, 64), ("l1_conv3", 512, 56, 56, 64, 256),
    ("l2_conv1", 512, 28, 28, 512, 128), ("l2_conv3", 512, 28, 28, 128, 512),
    ("l3_conv1", 512, 14, 14, 1024, 256), ("l3_conv3", 512, 14, 14, 256, 1024),
    ("l4_conv1", 512, 7, 7, 2048, 512), ("l4_conv3", 512, 7, 7, 512, 2048),
]


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, n, h, w, ci, co in SHAPES:
        x = torch.randn(n, ci, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(co, ci, device=dev) / ci ** 0.5).to(torch.bfloat16)
        arms = {"plain": lambda: _C.conv1x1_fwd(x, wt, None, None, False, False),
                "stats": lambda: _C.conv1x1_fwd(x, wt, None, None, False, True)}
        t = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                t[k].append(timeit(fn))
        byts = (n * h * w * (ci + co) + ci * co) * 2
        r = {"shape": name, "M": n * h * w, "K": ci, "N": co}
        for k, v in t.items():
            med = statistics.median(v)
            r[k + "_us"] = round(med, 1)
            r[k + "_TBps"] = round(byts / med / 1e6, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
