"""Isolate which part of a training step breaks HIP-graph capture."""
import os
import sys
import traceback

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29881")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
import distributed_compute_pytorch_amd as dcp  # noqa: E402
from distributed_compute_pytorch_amd.models import resnet18_like  # noqa: E402

dev = torch.device("cuda", 0)
dcp.distributed.init_process_group("rccl", device_id=0)


def attempt(name, fused, use_ddp, bwd, opt_kind, bench=True):
    torch.backends.cudnn.benchmark = bench
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        m = resnet18_like(num_classes=10, fused_bn=fused).to(dev).to(memory_format=torch.channels_last)
        net = dcp.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True) if use_ddp else m
        opt = None
        if opt_kind == "ours":
            opt = dcp.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
        elif opt_kind == "torch":
            opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, capturable=True) \
                if "capturable" in torch.optim.SGD.__init__.__code__.co_varnames else torch.optim.SGD(net.parameters(), lr=0.1)
    x = torch.randn(8, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)

    def step():
        if opt is not None:
            opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(net(x), y)
        if bwd:
            loss.backward()
        if opt is not None:
            opt.step()
        return loss

    try:
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = step()
        g.replay()
        torch.cuda.synchronize()
        print(f"[OK]   {name}", flush=True)
    except Exception as e:
        print(f"[FAIL] {name}: {type(e).__name__}: {str(e).splitlines()[0]}", flush=True)
        tb = traceback.format_exc().splitlines()
        print("\n".join(l for l in tb if "File" in l or "Error" in l)[-1500:], flush=True)
        torch.cuda.synchronize()


attempt("fwd only, stock BN, no ddp", False, False, False, None)
attempt("fwd+bwd, stock BN, no ddp", False, False, True, None)
attempt("fwd+bwd, stock BN, no ddp, cudnn.benchmark=0", False, False, True, None, bench=False)
attempt("fwd only, fused BN, no ddp", True, False, False, None)
attempt("fwd+bwd, fused BN, no ddp", True, False, True, None)
attempt("fwd+bwd+opt(ours), fused, no ddp", True, False, True, "ours")
attempt("fwd+bwd, fused, ddp", True, True, True, None)
attempt("full step ours", True, True, True, "ours")
