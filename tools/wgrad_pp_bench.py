"""Weight-gradient GEMMs: the 8-wave ping-pong kernel (wgrad_pp.hip) vs the
128 x 128 split-M ring (gemm.hip, gemm_tune wg_pp=0) vs hipBLASLt (torch.mm
with an fp32 output), interleaved rounds in one process (median us, TF/s).

    python tools/wgrad_pp_bench.py [--rounds 5] [--iters 10] [--only linear|conv]
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

LINEAR = [  # (name, M, N1 = out, N2 = in)
    ("gpt2_qkv", 8192, 2304, 768), ("gpt2_proj", 8192, 768, 768), ("gpt2_fc", 8192, 3072, 768),
    ("gpt2_fc2", 8192, 768, 3072), ("gpt2_head", 8192, 50304, 768),
    ("bert_qkv", 16384, 2304, 768), ("bert_fc", 16384, 3072, 768), ("bert_fc2", 16384, 768, 3072),
    ("bert_head", 2560, 30528, 768),
    ("rn_l3_c1", 100352, 256, 1024), ("rn_l3_c3", 100352, 1024, 256), ("rn_l4_c1", 25088, 512, 2048),
    ("rn_l4_c3", 25088, 2048, 512), ("rn_l3_ds", 100352, 1024, 512), ("rn_l4_ds", 25088, 2048, 1024),
]
CONV = [  # (name, N, H, W, Cin, Cout, k, stride, pad)
    ("rn_l3_3x3", 512, 14, 14, 256, 256, 3, 1, 1), ("rn_l3_3x3_s2", 512, 28, 28, 256, 256, 3, 2, 1),
    ("rn_l4_3x3", 512, 7, 7, 512, 512, 3, 1, 1), ("rn_l4_3x3_s2", 512, 14, 14, 512, 512, 3, 2, 1),
]


def timeit(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def run(name, flops, cands, rounds, iters):
    t = {k: [] for k in cands}
    for _ in range(rounds):
        for k, (pre, fn) in cands.items():
            pre()
            t[k].append(timeit(fn, iters))
    _C.gemm_tune("wg_pp", 1)
    r = {"shape": name, "GFLOP": round(flops / 1e9, 1)}
    for k, v in t.items():
        med = statistics.median(v)
        r[k + "_us"] = round(med, 1)
        r[k + "_TFps"] = round(flops / med / 1e6, 1)
    print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default=None)
    ap.add_argument("--names", default=None, help="comma-separated subset of the shape names")
    ap.add_argument("--xent-data", action="store_true",
                    help="gy as a cross-entropy logits gradient (softmax - onehot) / M instead of N(0, 1)")
    ap.add_argument("--multi", type=int, default=0,
                    help="also time the multi-segment launch over this many row segments of M rows each")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    pp = lambda: _C.gemm_tune("wg_pp", 1)  # noqa: E731
    ring = lambda: _C.gemm_tune("wg_pp", 0)  # noqa: E731
    if a.only in (None, "linear"):
        for name, m, n1, n2 in LINEAR:
            if a.names and name not in a.names.split(","):
                continue
            if a.xent_data:
                z = torch.randn(m, n1, device=dev) * 2.0
                g = torch.softmax(z, 1)
                g[torch.arange(m, device=dev), torch.randint(0, n1, (m,), device=dev)] -= 1.0
                g = (g / m).to(torch.bfloat16)
                del z
            else:
                g = torch.randn(m, n1, device=dev).to(torch.bfloat16)
            x = torch.randn(m, n2, device=dev).to(torch.bfloat16)
            acc = torch.zeros(n1, n2, device=dev)
            cands = {"pp": (pp, lambda: _C.conv1x1_wgrad(g, x)),
                     "pp_acc": (pp, lambda: _C.conv1x1_wgrad(g, x, accumulate_into=acc)),
                     "ring": (ring, lambda: _C.conv1x1_wgrad(g, x)),
                     "blas_acc": (pp, lambda: torch.addmm(acc, g.t(), x, out_dtype=torch.float32))}
            if a.multi > 1:
                gs = [g] + [g.clone() for _ in range(a.multi - 1)]
                xs = [x] + [x.clone() for _ in range(a.multi - 1)]
                gcat, xcat = torch.cat(gs), torch.cat(xs)
                cands[f"multi{a.multi}"] = (pp, lambda: _C.conv1x1_wgrad_multi(gs, xs, accumulate_into=acc))
                cands[f"cat{a.multi}"] = (pp, lambda: _C.conv1x1_wgrad(gcat, xcat, accumulate_into=acc))
            run(name, 2.0 * m * n1 * n2, cands, a.rounds, a.iters)
            del g, x, acc
            if a.multi > 1:
                del gs, xs, gcat, xcat
    if a.only in (None, "conv"):
        for name, n, h, w, ci, co, k, s, p in CONV:
            x = torch.randn(n, ci, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
            gy = torch.randn(n, co, ho, wo, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            cands = {"pp": (pp, lambda: _C.conv_wgrad(gy, x, k, k, s, p)),
                     "ring": (ring, lambda: _C.conv_wgrad(gy, x, k, k, s, p))}
            run(name, 2.0 * n * ho * wo * co * ci * k * k, cands, a.rounds, a.iters)


if __name__ == "__main__":
    main()
