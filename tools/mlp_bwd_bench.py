"""The MLP backward's GELU data gradient at the GPT-2 / BERT shapes: the ring
(gemm.hip EPI 10/11) and ping-pong (gemm_pp.hip EPI 4/5) fused kernels vs the
unfused hipBLASLt dgrad + gelu_bwd pass.

    python tools/mlp_bwd_bench.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


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
    for name, M, N1, N2, tanh in (("gpt2", 8192, 3072, 768, True), ("bert", 16384, 3072, 768, False)):
        gy = torch.randn(M, N2, device=dev).to(torch.bfloat16)
        w2 = (torch.randn(N2, N1, device=dev) / N1 ** 0.5).to(torch.bfloat16)
        w2t = w2.t().contiguous()
        h = torch.randn(M, N1, device=dev).to(torch.bfloat16)
        r = {"model": name, "M": M, "N1": N1, "N2": N2}
        for k, fn in (("ring", lambda: _C.linear_dgrad_gelu(gy, w2t, h, tanh)),
                      ("pp", lambda: _C.linear_dgrad_gelu(gy, w2t, h, tanh, pp=True)),
                      ("pp_dgrad_only", lambda: _C.gemm_pp(gy, w2t, None, 0)),
                      ("blas_unfused", lambda: _C.gelu_bwd(torch.mm(gy, w2), h, tanh, True))):
            r[k + "_us"] = round(timeit(fn, a.iters), 1)
        # the forward's GELU epilogue on fc (K = N2 -> N1)
        x = torch.randn(M, N2, device=dev).to(torch.bfloat16)
        w1 = (torch.randn(N1, N2, device=dev) / N2 ** 0.5).to(torch.bfloat16)
        b1 = torch.randn(N1, device=dev)
        mode = 1 if tanh else 2
        for k, fn in (("pp_fwd_bias", lambda: _C.gemm_pp(x, w1, b1, 0)),
                      ("pp_fwd_gelu", lambda: _C.gemm_pp(x, w1, b1, mode)),
                      ("ring_fwd_gelu", lambda: _C.linear_fwd(x, w1, b1, mode)),
                      ("gelu_bwd_pass", lambda: _C.gelu_bwd(gy.new_empty(M, N1).normal_(), h, tanh, True))):
            r[k + "_us"] = round(timeit(fn, a.iters), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
