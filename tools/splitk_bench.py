"""Split-K sweep of the ping-pong GEMM on the shapes whose 256 x 256 tiles
leave CUs idle (GPT-2 / BERT LM-head data gradient, the N = 768 GEMMs):
forced split counts vs the time model's pick vs hipBLASLt, interleaved
rounds in one process (median us). One JSON line per shape.

    python tools/splitk_bench.py [--rounds 5] [--iters 10] [--splits 1,2,4,5,8]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402

SHAPES = [("gpt2_head_dgrad", 8192, 768, 50304), ("bert_head_dgrad", 16384, 768, 30592),
          ("gpt2_fc2_dgrad", 8192, 768, 3072), ("gpt2_qkv_dgrad", 8192, 768, 2304)]


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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", default="1,2,3,4,5,6,8")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    splits = [int(s) for s in a.splits.split(",")]
    for name, M, N, K in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16)

        def pp(S):
            C.gemm_tune("pp_sk_force", S)
            C.gemm_tune("pp_sk", 1 if S != 1 else 0)
            return C.gemm_pp(x, w)

        ops = {f"S{S}": (lambda S=S: pp(S)) for S in splits}
        ops["auto"] = lambda: pp(0)
        ops["blas"] = lambda: torch.mm(x, w.t())
        ts = {k: [] for k in ops}
        for _ in range(a.rounds):
            for k, f in ops.items():
                ts[k].append(timeit(f, a.iters))
        C.gemm_tune("pp_sk_force", 0)
        C.gemm_tune("pp_sk", 1)
        row = {"shape": name, "M": M, "N": N, "K": K, "auto_S": C.gemm_pp_splitk(M, N, K)}
        row.update({k + "_us": round(statistics.median(v), 1) for k, v in ts.items()})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
