"""Op-level HIP-graph replay check: capture one op, replay it several times,
compare every output with the eager op on the same inputs. Finds ops whose
captured form depends on state outside the graph (e.g. an accumulator whose
zeroing was not captured).

    python tools/graph_op_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
cl = torch.channels_last
x = torch.randn(8, 64, 16, 16, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
w1 = torch.randn(64, 64, device=dev).to(torch.bfloat16)
w3 = torch.randn(64, 3, 3, 64, device=dev).to(torch.bfloat16)
g = torch.rand(64, device=dev) + 0.5
b = torch.randn(64, device=dev)


def ops():
    return {
        "conv1x1 stats": lambda: _C.conv1x1_fwd(x, w1, None, None, False, True),
        "conv_fwd stats": lambda: _C.conv_fwd(x, w3, 3, 3, 1, 1, True),
        "bn_act_fwd": lambda: _C.bn_act_fwd(x, g, b, None, None, None, True, 0.1, 1e-5, True, None, None)[:3],
        "memset": lambda: [torch.zeros(128, device=dev).add_(1.0)],
    }


def flat(out):
    return [t.float().clone() for t in out if torch.is_tensor(t) and t.numel()]


for name, fn in ops().items():
    mode = os.environ.get("MODE", "side")
    ref = flat(fn())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s, capture_error_mode="thread_local"):
        out = fn()
    errs = []
    for i in range(3):
        gr.replay()
        torch.cuda.synchronize()
        errs.append(max(float((a - r).abs().max() / r.abs().max().clamp_min(1e-12)) for a, r in zip(flat(out), ref)))
    print(f"{name:16s} replay max rel err: " + " ".join(f"{e:.2e}" for e in errs), flush=True)
