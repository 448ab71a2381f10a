"""Host/GPU timing breakdown of one flash-attention fwd+bwd at the BERT shape
(diagnoses tools/attn_bench.py's BERT fwd+bwd outlier)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd.ops.attention import flash_attn  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for name, B, T, H, causal, p in [("bert", 32, 512, 12, False, 0.1), ("gpt2", 8, 1024, 12, True, 0.1),
                                     ("bert-nodrop", 32, 512, 12, False, 0.0)]:
        C = H * 64
        q, k, v, do = (torch.randn(B, T, C, device=dev, dtype=torch.bfloat16) for _ in range(4))
        qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
        for it in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            o = flash_attn(qa, ka, va, H, causal, p)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            o.backward(do)
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            print(f"{name} it{it}: fwd host {1e3*(t1-t0):.2f} ms, fwd sync {1e3*(t2-t1):.2f}, "
                  f"bwd host {1e3*(t3-t2):.2f}, bwd sync {1e3*(t4-t3):.2f}", flush=True)
        # without grad accumulation into the leaves
        for it in range(3):
            qb, kb, vb = (t.clone().requires_grad_(True) for t in (q, k, v))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            flash_attn(qb, kb, vb, H, causal, p).backward(do)
            torch.cuda.synchronize()
            print(f"{name} fresh-leaves it{it}: {1e3*(time.perf_counter()-t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
