"""A few launches of the GEMM families the VERDICT asks PMC evidence for, one
shape each, for rocprofv3 --pmc (tools/gemm_pmc.sh):
  rn50 L3 conv1 forward  [100352 x 1024] · [256 x 1024]ᵀ  (+ BN sums epilogue)
  rn50 L3 conv3 forward  [100352 x 256]  · [1024 x 256]ᵀ  (+ BN sums epilogue)
  rn50 L3 conv1 wgrad    dW [256 x 1024] over 100352 rows
  gpt2 fc wgrad          dW [3072 x 768] over 8192 rows
  bert fc1 forward on the ping-pong GEMM [16384 x 768] · [3072 x 768]ᵀ (+ bias)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*shape, scale=1.0):
    return ((torch.rand(*shape, device=dev, generator=g) * 2 - 1) * scale).to(torch.bfloat16)


x1 = rnd(512, 14, 14, 1024).permute(0, 3, 1, 2)   # channels_last [512, 1024, 14, 14]
w1 = rnd(256, 1024, scale=1024 ** -0.5)
x3 = rnd(512, 14, 14, 256).permute(0, 3, 1, 2)
w3 = rnd(1024, 256, scale=256 ** -0.5)
gy1 = rnd(100352, 256)
xa = rnd(100352, 1024)
gt = rnd(8192, 3072)
xt = rnd(8192, 768)
xb = rnd(16384, 768)
wb = rnd(3072, 768, scale=768 ** -0.5)
bb = torch.zeros(3072, device=dev)
for _ in range(3):
    C.conv1x1_fwd(x1, w1, None, None, False, True)
    C.conv1x1_fwd(x3, w3, None, None, False, True)
    C.conv1x1_wgrad(gy1, xa)
    C.conv1x1_wgrad(gt, xt)
    C.gemm_pp(xb, wb, bb, 0)
torch.cuda.synchronize()
print("done")
