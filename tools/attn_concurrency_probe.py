"""Would running the attention backward's dQ and dK/dV kernels concurrently
help? Proxy: two independent backward passes (BERT / GPT-2 shape, dropout
0.1) on two streams at once vs one after the other, graph-replayed.

    python tools/attn_concurrency_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd.ops.attention import flash_attn  # noqa: E402


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    for name, B, T, H, causal in (("bert", 32, 512, 12, False), ("gpt2", 8, 1024, 12, True)):
        C = H * 64
        probs = []
        for _ in range(2):
            q, k, v, do = (torch.randn(B, T, C, device=dev, dtype=torch.bfloat16) for _ in range(4))
            qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
            probs.append((qa, ka, va, do))

        def one(p):
            qa, ka, va, do = p
            torch.autograd.grad(flash_attn(qa, ka, va, H, causal, 0.1), (qa, ka, va), do)

        side = torch.cuda.Stream()

        def serial():
            one(probs[0])
            one(probs[1])

        def concurrent():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                one(probs[1])
            one(probs[0])
            cur.wait_stream(side)

        r = {"case": name, "one_us": round(timed(lambda: one(probs[0])), 1),
             "serial_two_us": round(timed(serial), 1), "concurrent_two_us": round(timed(concurrent), 1)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
