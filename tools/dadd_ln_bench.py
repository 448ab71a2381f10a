"""Residual dropout + LayerNorm at the GPT-2 (fp32 residual, 8,192 rows) and
BERT (bf16 residual, 16,384 rows) shapes: the fused LnDropAdd kernels vs
dropout_add then the LayerNorm, forward and backward (HIP-event time).

    python tools/dadd_ln_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def timeit(fn, iters=20):
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
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    for name, M, rdt in (("gpt2", 8192, torch.float32), ("bert", 16384, torch.bfloat16)):
        D = 768
        br = torch.randn(M, D, device=dev).to(bf)
        res = torch.randn(M, D, device=dev).to(rdt)
        w, b = torch.ones(D, device=dev), torch.zeros(D, device=dev)
        out_dt = bf if rdt == torch.float32 else None
        r = {"case": name}
        r["unfused_fwd_us"] = round(timeit(lambda: _C.layer_norm_fwd(_C.dropout_fwd(br, res, 0.1, 1, 0, None, None), w,
                                                                       b, 1e-5, out_dt)), 1)
        r["fused_fwd_us"] = round(timeit(lambda: _C.layer_norm_fwd(res, w, b, 1e-5, out_dt, branch=br, p=0.1, seed=1)), 1)
        y, mu, rs, x = _C.layer_norm_fwd(res, w, b, 1e-5, out_dt, branch=br, p=0.1, seed=1)
        dy = torch.randn(M, D, device=dev).to(bf)
        g2 = torch.randn(M, D, device=dev).to(rdt)
        r["unfused_bwd_us"] = round(timeit(lambda: _C.dropout_fwd(
            _C.layer_norm_bwd(dy, x, w, b, mu, rs, grad_residual=g2)[0], None, 0.1, 1, 0, bf, None)), 1)
        r["fused_bwd_us"] = round(timeit(lambda: _C.layer_norm_bwd(dy, x, w, b, mu, rs, grad_residual=g2, drop_p=0.1,
                                                                   drop_seed=1, branch_grad=True)), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
