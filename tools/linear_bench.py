"""Transformer Linear GEMMs at the BERT-base (b32 x 512) / GPT-2-small (b8 x 1024)
shapes: our gemm_nt with the bias (+GELU) epilogue (_C.linear_fwd) and the
data-gradient GEMM (_C.conv1x1_dgrad) vs hipBLASLt through torch, under each
requested gemm_tune setting. One JSON line per (shape, op).

    python tools/linear_bench.py [--iters 20] [--tune lin_big=0 lin_big=1 lin_big=2 nt_big=2]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402

SHAPES = [("bert", 16384, 768, 768), ("bert", 16384, 768, 3072), ("bert", 16384, 3072, 768),
          ("gpt2", 8192, 768, 2304), ("gpt2", 8192, 768, 768), ("gpt2", 8192, 768, 3072), ("gpt2", 8192, 3072, 768)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


WG_VARIANTS = ["wg_cap=0", "wg_cap=1", "wg_cap=4"]


def wgrad(model, M, K, N, x, gy, a):
    """dW [N, K] = gyᵀ x (fp32) — our split-M wgrad under each slab plan vs hipBLASLt."""
    fl = 2 * M * N * K
    rec = {"model": model, "M": M, "K": K, "N": N, "op": "wgrad"}
    ref = None
    for kv in a.wg_variants:
        olds = {}
        for e in kv.split("+"):
            k, v = e.split("=")
            olds[k] = _C.gemm_tune_get(k)
            _C.gemm_tune(k, int(v))
        out = _C.conv1x1_wgrad(gy, x)
        if ref is None:
            ref = out
        else:
            rec[kv + "_maxdiff"] = float((out - ref).abs().max())
        us = timeit(lambda: _C.conv1x1_wgrad(gy, x), a.iters)
        for k, v in olds.items():
            _C.gemm_tune(k, v)
        rec[kv], rec[kv + "_TF"] = round(us, 1), round(fl / us / 1e6, 1)
    us = timeit(lambda: torch.mm(gy.t(), x, out_dtype=torch.float32), a.iters)
    rec["blas"], rec["blas_TF"] = round(us, 1), round(fl / us / 1e6, 1)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--wgrad-only", action="store_true")
    ap.add_argument("--wg-variants", nargs="*", default=WG_VARIANTS, help="gemm_tune settings of the wgrad A/B")
    ap.add_argument("--wgrad3", action="store_true", help="ResNet-50 3x3 weight gradients under each --tune entry")
    ap.add_argument("--tune", nargs="*", default=["lin_big=0", "lin_big=1", "lin_big=2"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    if a.wgrad3:
        for hw, c in [(28, 128), (14, 256), (7, 512)]:
            n = 512
            xi = torch.randn(n, c, hw, hw, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
            gi = torch.randn(n, c, hw, hw, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
            fl = 2 * n * hw * hw * c * 9 * c
            rec = {"model": f"resnet3x3_{hw}", "C": c, "op": "wgrad3"}
            ref = None
            for kv in a.tune:
                olds = {}
                for e in kv.split("+"):
                    k, v = e.split("=")
                    olds[k] = _C.gemm_tune_get(k)
                    _C.gemm_tune(k, int(v))
                out = _C.conv_wgrad(gi, xi, 3, 3, 1, 1)
                if ref is None:
                    ref = out
                else:
                    rec[kv + "_maxrel"] = float((out - ref).abs().max() / ref.abs().max())
                us = timeit(lambda: _C.conv_wgrad(gi, xi, 3, 3, 1, 1), a.iters)
                for k, v in olds.items():
                    _C.gemm_tune(k, v)
                rec[kv], rec[kv + "_TF"] = round(us, 1), round(fl / us / 1e6, 1)
            print(json.dumps(rec), flush=True)
        return
    if a.wgrad_only:
        for hw, ci, co in [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
                           (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]:
            M = 512 * hw * hw
            x = torch.randn(M, ci, device=dev).to(bf)
            gy = torch.randn(M, co, device=dev).to(bf)
            wgrad(f"resnet{hw}", M, ci, co, x, gy, a)
        for model, M, K, N in SHAPES:
            if N >= K or model == "gpt2":
                wgrad(model, M, K, N, torch.randn(M, K, device=dev).to(bf), torch.randn(M, N, device=dev).to(bf), a)
        return
    for model, M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(bf)
        wt = w.t().contiguous()
        b = torch.randn(N, device=dev)
        gy = torch.randn(M, N, device=dev).to(bf)
        for gelu in ([0, 2] if N > K else [0]):
            rec = {"model": model, "M": M, "K": K, "N": N, "op": "fwd" + ("_gelu" if gelu else "")}
            fl = 2 * M * N * K
            for kv in a.tune:
                olds = {}
                for e in kv.split("+"):
                    k, v = e.split("=")
                    olds[k] = _C.gemm_tune_get(k)
                    _C.gemm_tune(k, int(v))
                us = timeit(lambda: _C.linear_fwd(x, w, b, gelu), a.iters)
                for k, v in olds.items():
                    _C.gemm_tune(k, v)
                rec[kv] = round(us, 1)
                rec[kv + "_TF"] = round(fl / us / 1e6, 1)
            b16 = b.to(bf)
            blas = (lambda: F.gelu(F.linear(x, w, b16))) if gelu else (lambda: F.linear(x, w, b16))
            us = timeit(blas, a.iters)
            rec["blas"], rec["blas_TF"] = round(us, 1), round(fl / us / 1e6, 1)
            print(json.dumps(rec), flush=True)
        rec = {"model": model, "M": M, "K": N, "N": K, "op": "dgrad"}
        for kv in ["nt_big=4", "nt_big=2", "nt_big=2+big_pipe=1"]:
            olds = {}
            for e in kv.split("+"):
                k, v = e.split("=")
                olds[k] = _C.gemm_tune_get(k)
                _C.gemm_tune(k, int(v))
            us = timeit(lambda: _C.conv1x1_dgrad(gy, wt), a.iters)
            for k, v in olds.items():
                _C.gemm_tune(k, v)
            rec[kv], rec[kv + "_TF"] = round(us, 1), round(fl / us / 1e6, 1)
        us = timeit(lambda: gy @ w, a.iters)
        rec["blas"], rec["blas_TF"] = round(us, 1), round(fl / us / 1e6, 1)
        print(json.dumps(rec), flush=True)
        wgrad(model, M, K, N, x, gy, a)


if __name__ == "__main__":
    main()
