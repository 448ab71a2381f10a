"""Linear weight gradient dW[N1, N2] = g[M, N1]ᵀ · x[M, N2] (fp32 out) at the
BERT-base / GPT-2-small shapes: our split-M MFMA wgrad (gemm.hip) vs
hipBLASLt through torch.mm (fp32 out, and bf16 out + cast).

    python tools/linear_wgrad_bench.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402

SHAPES = [  # (M, N1 = out features, N2 = in features)
    (16384, 768, 768), (16384, 2304, 768), (16384, 3072, 768), (16384, 768, 3072),
    (8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072),
]


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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for m, n1, n2 in SHAPES:
        g = torch.randn(m, n1, device=dev).to(torch.bfloat16)
        x = torch.randn(m, n2, device=dev).to(torch.bfloat16)
        flops = 2.0 * m * n1 * n2
        r = {"M": m, "N1": n1, "N2": n2}
        acc = torch.zeros(n1, n2, device=dev)
        for name, fn in (("ours", lambda: _C.conv1x1_wgrad(g, x)),
                         ("ours_acc", lambda: _C.conv1x1_wgrad(g, x, accumulate_into=acc)),
                         ("addmm_fp32_acc", lambda: torch.addmm(acc, g.t(), x, out_dtype=torch.float32)),
                         ("mm_fp32out", lambda: torch.mm(g.t(), x, out_dtype=torch.float32)),
                         ("mm_bf16_cast", lambda: torch.mm(g.t(), x).float())):
            try:
                us = timeit(fn, a.iters)
                r[name + "_us"] = round(us, 1)
                r[name + "_TFps"] = round(flops / us / 1e6, 1)
            except Exception as ex:  # noqa: BLE001
                r[name + "_err"] = str(ex)[:80]
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
