"""A few launches of one GEMM for rocprofv3 --pmc (gemm_pp single-tile kernel,
gemm_pp persistent, our 128x128 ring, hipBLASLt) at one shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 4096, 4096)))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
b = torch.zeros(N, device=dev)
for _ in range(3):
    C.gemm_tune("pp_v1", 1)
    C.gemm_pp(x, w)
    C.gemm_tune("pp_v1", 0)
    C.gemm_pp(x, w)
    C.linear_fwd(x, w, b, 0)
    torch.mm(x, w.t())
torch.cuda.synchronize()
print("done", M, N, K)
