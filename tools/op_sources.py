"""Which Python lines issue the small ATen copies / fills of a training step?

Runs the bench workload (our DDP + fused optimizer, one rank) for a few
warm-up steps, then records `--steps` steps under a TorchDispatchMode (
with Python stacks) and prints, per step, how often each copy / fill /
zeros-like ATen op was called and from which line of this package.

    python tools/op_sources.py --model bert [--steps 2]
"""
import argparse
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = {"aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::clone",
       "aten::contiguous", "aten::_to_copy", "aten::cat", "aten::index_put_", "aten::index_add_",
       "aten::embedding_dense_backward", "aten::new_zeros"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29000 + os.getpid() % 1000))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dev = torch.device("cuda", 0)
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd import workloads

    wl = workloads.build(a.model, dev, fused=True)
    dcp.distributed.init_process_group("rccl", device_id=0)
    # the bench's DDP settings that change which ops run (bench.py)
    kw = {"defer_accum_wgrad": True} if wl.accum > 1 else {}
    ddp = dcp.parallel.DistributedDataParallel(wl.model, device_ids=[0], gradient_as_bucket_view=True, **kw)
    opt = wl.make_optimizer(ddp.parameters())
    step = workloads.make_step(wl, ddp, opt)
    for _ in range(6):
        step()
    torch.cuda.synchronize()
    import traceback

    from torch.utils._python_dispatch import TorchDispatchMode

    pkg = os.path.dirname(os.path.abspath(dcp.__file__))
    cnt = Counter()

    class Spy(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = "aten::" + func.__name__.split(".")[0]
            if name in OPS:
                where = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if pkg in fr.filename or fr.filename.endswith("bench.py"):
                        where = f"{fr.filename.replace(pkg + '/', '')}:{fr.lineno} {fr.name}"
                        break
                cnt[(name, where)] += 1
            return func(*args, **(kwargs or {}))

    with Spy():
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    # the backward runs on the autograd device thread, outside the mode: the
    # profiler's parent chain (autograd node / op names) names those callers
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    chains = Counter()
    for e in prof.events():
        if e.name not in ("aten::copy_", "aten::fill_", "aten::zero_"):
            continue
        names, p = [], e.cpu_parent
        while p is not None and len(names) < 4:
            names.append(p.name)
            p = p.cpu_parent
        chains[(e.name, " < ".join(names))] += 1
    print(f"# {a.model}: copy / fill ops per step by profiler parent chain")
    for (n, w), c in chains.most_common(a.top):
        print(f"{c / a.steps:8.1f}  {n:14s} {w[:150]}")
    # every ATen op that launched a non-dcp GPU kernel, with its parent chain
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof2:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    launches = Counter()
    for e in prof2.events():
        ks = [k for k in getattr(e, "kernels", []) if not k.name.startswith("dcp::")]
        if not ks or not e.name.startswith("aten::"):
            continue
        names, p = [], e.cpu_parent
        while p is not None and len(names) < 3:
            names.append(p.name)
            p = p.cpu_parent
        launches[(e.name, ks[0].name[:40], " < ".join(names))] += len(ks)
    print(f"# {a.model}: non-dcp GPU kernels per step by launching ATen op and parent chain")
    for (n, k, w), c in launches.most_common(a.top):
        print(f"{c / a.steps:8.1f}  {n:22s} {k:40s} {w[:120]}")
    print(f"# {a.model}: ATen copy / fill ops per step and the first frame in the package")
    for (n, w), c in cnt.most_common(a.top):
        print(f"{c / a.steps:8.1f}  {n:28s} {w}")
    dcp.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
