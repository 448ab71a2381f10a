"""Embedding weight-gradient variants at the BERT / GPT-2 shapes: ATen
index_add_ (fp32 atomics) vs a one-hot GEMM for tiny vocabularies (BERT's
2-row token-type table, where every row of the batch hits the same 2 x 768
addresses).

    python tools/emb_bench.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    D = 768
    for name, V, M, kind in (("bert_word", 30522, 16384, "rand"), ("bert_type_zeros", 2, 16384, "zeros"),
                             ("bert_type_rand", 2, 16384, "rand"), ("gpt2_wte", 50257, 8192, "rand")):
        idx = torch.randint(0, V, (M,), device=dev) if kind == "rand" else torch.zeros(M, dtype=torch.long, device=dev)
        g = torch.randn(M, D, device=dev)
        gw = torch.zeros(V, D, device=dev)
        r = {"case": name, "index_add_us": round(timeit(lambda: gw.index_add_(0, idx, g)), 1)}
        if V <= 8:
            import distributed_compute_pytorch_amd  # noqa: F401
            from distributed_compute_pytorch_amd._ext import C as _C

            r["small_kernel_us"] = round(timeit(lambda: _C.embedding_small_bwd(idx, g, gw)), 1)
        if V <= 16:
            r["onehot_mm_us"] = round(timeit(lambda: F.one_hot(idx, V).to(torch.float32).t() @ g), 1)
            r["onehot_addmm_us"] = round(timeit(lambda: gw.addmm_(F.one_hot(idx, V).to(torch.float32).t(), g)), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
