"""Attention fwd / fwd+bwd at the BERT-base (B32 T512 H12, dropout 0.1) and
GPT-2-small (B8 T1024 H12 causal, dropout 0.1) shapes: our MFMA flash
attention vs torch scaled_dot_product_attention (aotriton on ROCm).

    python tools/attn_bench.py [--iters 10] [--graph 1]

--graph 1 (default) times replays of a captured HIP graph of each call, so
the numbers are GPU time (the eager loop's autograd / launch overhead per
fwd+bwd, ~40-50 µs, exceeds the BERT-shape kernels' idle slack); --graph 0
times the eager calls.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd.ops.attention import flash_attn  # noqa: E402


GRAPH = True


def timeit(fn, iters):
    # three warm-up calls: the process's first two backward passes carry the
    # autograd engine's one-time start-up (0.7 s + 70 ms, tools/attn_diag.py)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    run = fn
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        run = g.replay
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", nargs="*", default=None, help="subset of bert gpt2 bert-nodrop gpt2-nodrop")
    ap.add_argument("--graph", type=int, default=1)
    a = ap.parse_args()
    global GRAPH
    GRAPH = bool(a.graph)
    dev = torch.device("cuda", 0)
    for name, B, T, H, causal, p in [("bert", 32, 512, 12, False, 0.1), ("gpt2", 8, 1024, 12, True, 0.1),
                                     ("bert-nodrop", 32, 512, 12, False, 0.0), ("gpt2-nodrop", 8, 1024, 12, True, 0.0)]:
        if a.cases and name not in a.cases:
            continue
        C = H * 64
        q, k, v, do = (torch.randn(B, T, C, device=dev, dtype=torch.bfloat16) for _ in range(4))
        qs, ks, vs = (t.view(B, T, H, 64).transpose(1, 2) for t in (q, k, v))
        fl = 4.0 * B * H * T * T * 64 * (0.5 if causal else 1.0)
        r = {"case": name, "graph": GRAPH}
        r["ours_fwd_us"] = timeit(lambda: flash_attn(q, k, v, H, causal, p), a.iters)
        r["sdpa_fwd_us"] = timeit(lambda: F.scaled_dot_product_attention(qs, ks, vs, dropout_p=p, is_causal=causal),
                                  a.iters)
        qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))

        # torch.autograd.grad: the gradients come back as new tensors, as in a
        # training step (where they feed the projection's backward) — a
        # .backward() here would add three [B, T, C] .grad accumulations
        # (~45 µs at the BERT shape) to every fwd+bwd
        def ours_fb():
            torch.autograd.grad(flash_attn(qa, ka, va, H, causal, p), (qa, ka, va), do)

        qsa, ksa, vsa = (t.clone().requires_grad_(True) for t in (qs, ks, vs))
        dos = do.view(B, T, H, 64).transpose(1, 2)

        def sdpa_fb():
            torch.autograd.grad(F.scaled_dot_product_attention(qsa, ksa, vsa, dropout_p=p, is_causal=causal),
                                (qsa, ksa, vsa), dos)

        r["ours_fwdbwd_us"] = timeit(ours_fb, a.iters)
        r["sdpa_fwdbwd_us"] = timeit(sdpa_fb, a.iters)
        r["ours_fwd_TFps"] = fl / (r["ours_fwd_us"] * 1e-6) / 1e12
        r["ours_fwdbwd_TFps"] = 3.5 * fl / (r["ours_fwdbwd_us"] * 1e-6) / 1e12
        print(json.dumps({kk: (round(vv, 1) if isinstance(vv, float) else vv) for kk, vv in r.items()}), flush=True)


if __name__ == "__main__":
    main()
