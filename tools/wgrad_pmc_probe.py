"""Launches of the weight-gradient kernels for rocprofv3 (kernel trace / PMC):
3 calls each of the ping-pong wgrad at the GPT-2 fc, BERT fc, GPT-2 LM-head
(one slab: no reduction) and ResNet layer-3 3x3 shapes, then the same shapes
on the ring kernel (gemm_tune wg_pp = 0).

    rocprofv3 --kernel-trace --stats -- python3 tools/wgrad_pmc_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lin = [(8192, 3072, 768), (16384, 3072, 768), (8192, 50304, 768)]
    ops = []
    for m, n1, n2 in lin:
        g = torch.randn(m, n1, device=dev).to(torch.bfloat16)
        x = torch.randn(m, n2, device=dev).to(torch.bfloat16)
        ops.append(lambda g=g, x=x: _C.conv1x1_wgrad(g, x))
    # GPT-2 fc over 4 deferred micro-steps (one multi-segment launch)
    gs = [torch.randn(8192, 3072, device=dev).to(torch.bfloat16) for _ in range(4)]
    xs = [torch.randn(8192, 768, device=dev).to(torch.bfloat16) for _ in range(4)]
    ops.append(lambda: _C.conv1x1_wgrad_multi(gs, xs))
    x = torch.randn(512, 256, 14, 14, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(512, 256, 14, 14, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ops.append(lambda: _C.conv_wgrad(gy, x, 3, 3, 1, 1))
    for v in (1, 0):
        _C.gemm_tune("wg_pp", v)
        for op in ops:
            for _ in range(3):
                op()
    torch.cuda.synchronize()
    _C.gemm_tune("wg_pp", 1)


if __name__ == "__main__":
    main()
