"""PMC probe: a few fwd+bwd calls of our flash attention at the GPT-2
(B8 T1024 H12 causal) and BERT (B32 T512 H12) shapes with dropout 0.1, for
tools/gemm_pmc.sh (PROBE=tools/attn_pmc_probe.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd.ops.attention import flash_attn  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for B, T, H, causal in ((8, 1024, 12, True), (32, 512, 12, False)):
        C = H * 64
        q, k, v, do = (torch.randn(B, T, C, device=dev, dtype=torch.bfloat16) for _ in range(4))
        qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
        for _ in range(3):
            flash_attn(qa, ka, va, H, causal, 0.1).backward(do)
        torch.cuda.synchronize()
    print("probe done")


if __name__ == "__main__":
    main()
