"""Why the LM-head weight gradient times differently in the model than in
tools/wgrad_pp_bench.py: the same call on (a) random operands, (b) the
cross-entropy gradient of random logits (what the model feeds it), each
with / without out_rows and accumulation, vs hipBLASLt — interleaved
rounds, median µs. One JSON line per arm.

    python tools/head_wgrad_probe.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def timeit(fn, iters=5):
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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, V, Vp, K = 8192, 50257, 50304, 768
    g = torch.Generator(device=dev).manual_seed(0)
    x2 = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    d_rand = torch.randn(M, Vp, device=dev, generator=g).to(torch.bfloat16)
    d_rand[:, V:] = 0
    logits = (torch.randn(M, Vp, device=dev, generator=g) * 2).to(torch.bfloat16)
    tg = torch.randint(0, V, (M,), device=dev, generator=g)
    _, lse = _C.cross_entropy_fwd(logits, tg, -100, 0.0, V)
    d_xent = _C.cross_entropy_bwd(logits.clone(), tg, lse, torch.full((1,), 1.0 / M, device=dev), -100, 0.0, V, True)
    acc_full = torch.zeros(Vp, K, device=dev)
    acc_v = torch.zeros(V, K, device=dev)
    arms = {}
    for dn, d in (("rand", d_rand), ("xent", d_xent)):
        arms[f"ours_{dn}"] = lambda d=d: _C.conv1x1_wgrad(d, x2)
        arms[f"ours_acc_{dn}"] = lambda d=d: _C.conv1x1_wgrad(d, x2, accumulate_into=acc_full)
        arms[f"ours_acc_rows_{dn}"] = lambda d=d: _C.conv1x1_wgrad(d, x2, accumulate_into=acc_v, out_rows=V)
        arms[f"blas_acc_{dn}"] = lambda d=d: torch.addmm(acc_v, d[:, :V].t(), x2, out_dtype=torch.float32, out=acc_v)
    ts = {k: [] for k in arms}
    for r in range(a.rounds):
        for k, f in arms.items():
            ts[k].append(timeit(f))
    for k, v in ts.items():
        print(json.dumps({"arm": k, "median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1)}), flush=True)


if __name__ == "__main__":
    main()
