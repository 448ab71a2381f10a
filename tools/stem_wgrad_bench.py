"""ResNet-50 stem weight gradient (7x7/2, 3->64, batch 512 at 224²) on our
split-M MFMA kernel: one 64 x 256 tile per slab (gemm_tune stem_wide=1) vs two
64 x 128 tiles (0), interleaved rounds, median us.

    python tools/stem_wgrad_bench.py [--rounds 5] [--iters 20] [--json out.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N, H, W = a.batch, 224, 224
    x = torch.randn(N, 3, H, W, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, 64, H // 2, W // 2, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xp, _ = C.stem_prep(x, False)
    res = {0: [], 1: []}
    outs = {}
    for _ in range(a.rounds):
        for wide in (1, 0):
            C.gemm_tune("stem_wide", wide)
            res[wide].append(timeit(lambda: C.stem_conv_wgrad(dy, xp, H, W), a.iters))
            outs[wide] = C.stem_conv_wgrad(dy, xp, H, W)
    C.gemm_tune("stem_wide", 1)
    diff = float((outs[1] - outs[0]).abs().max() / outs[0].abs().max())
    row = {"case": f"stem wgrad b{N}", "wide_us": round(statistics.median(res[1]), 1),
           "narrow_us": round(statistics.median(res[0]), 1), "rel_maxdiff": diff}
    print(json.dumps(row))
    if a.json:
        with open(a.json, "a") as f:
            f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
