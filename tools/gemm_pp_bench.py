"""Ping-pong 256x256 GEMM (gemm_pp) vs our 128x128 ring (linear_fwd / conv1x1
forward) vs hipBLASLt (torch.mm) on the transformer Linear and ResNet-50 1x1
shapes, random operands, interleaved rounds in one process (median us, TF/s).

    python tools/gemm_pp_bench.py [--rounds 5] [--iters 20] [--json out.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402

SHAPES = [  # (name, M, N, K)
    ("bert qkv/o 768->768", 16384, 768, 768), ("bert fc1 768->3072", 16384, 3072, 768),
    ("bert fc2 3072->768", 16384, 768, 3072), ("bert dgrad fc1 3072->768", 16384, 768, 3072),
    ("gpt2 c_attn 768->2304", 8192, 2304, 768), ("gpt2 fc 768->3072", 8192, 3072, 768),
    ("gpt2 proj 3072->768", 8192, 768, 3072), ("gpt2 attn-proj 768->768", 8192, 768, 768),
    ("gpt2 dgrad qkv 2304->768", 8192, 768, 2304), ("gpt2 lmhead 768->50304", 8192, 50304, 768),
    ("square 4096", 4096, 4096, 4096), ("square 8192", 8192, 8192, 8192),
    ("rn50 56x56 64->256", 512 * 56 * 56, 256, 64), ("rn50 28x28 512->128", 512 * 28 * 28, 128, 512),
    ("rn50 14x14 256->1024", 512 * 14 * 14, 1024, 256), ("rn50 14x14 1024->256", 512 * 14 * 14, 256, 1024),
    ("rn50 7x7 512->2048", 512 * 7 * 7, 2048, 512), ("rn50 7x7 2048->512", 512 * 7 * 7, 512, 2048),
]


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
    ap.add_argument("--json", default=None)
    ap.add_argument("--quick", action="store_true", help="skip the persistent variants")
    ap.add_argument("--names", default=None, help="comma-separated substrings of the shape names to run")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = open(a.json, "a") if a.json else None
    for name, M, N, K in SHAPES:
        if a.names and not any(t in name for t in a.names.split(",")):
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = torch.zeros(N, device=dev)
        def pp(stage, v1=1, bias=None, tile=1, ns=4):
            C.gemm_tune("pp_pq_ns", ns)
            C.gemm_tune("pp_stage", stage)
            C.gemm_tune("pp_v1", v1)
            C.gemm_tune("pp_tile", tile)  # 1: 256 x 256, 2: 128 x 192 (gemm_pq.hip)
            C.gemm_tune("pp_sk", 0)
            return C.gemm_pp(x, w, bias)

        ops = {"pp": lambda: pp(1), "blas": lambda: torch.mm(x, w.t())}
        if not a.quick:
            ops["pp_persist"] = lambda: pp(1, 0)
            ops["pp_persist_regepi"] = lambda: pp(0, 0)
        if N % 8 == 0:
            ops["pq"] = lambda: pp(1, tile=2)
            ops["pq3"] = lambda: pp(1, tile=2, ns=3)
            ops["pq_bias"] = lambda: pp(1, 1, b, tile=2)
        if N <= 7168:
            ops["pp_bias"] = lambda: pp(1, 1, b)
        if N % 64 == 0 and K <= 4096:
            ops["ring128"] = lambda: C.linear_fwd(x, w, b, 0)
        ref = torch.mm(x, w.t())
        rel = 0.0
        for v in [f for k, f in ops.items() if k.startswith("p") and "bias" not in k]:
            y = v()[0]
            rel = max(rel, float((y.float() - ref.float()).norm() / ref.float().norm()))
        ts = {k: [] for k in ops}
        for r in range(a.rounds):
            for k in (list(ops)[r % len(ops):] + list(ops)[:r % len(ops)]):
                ts[k].append(timeit(ops[k], a.iters))
        fl = 2.0 * M * N * K
        rec = {"shape": name, "M": M, "N": N, "K": K, "rel_err_vs_blas": round(rel, 5)}
        for k, v in ts.items():
            med = statistics.median(v)
            rec[k + "_us"] = round(med, 1)
            rec[k + "_TF"] = round(fl / med / 1e6, 1)
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
        del x, w, y, ref


if __name__ == "__main__":
    main()
