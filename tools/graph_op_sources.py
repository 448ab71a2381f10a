"""Which Python lines / autograd nodes issue the ATen copies, adds and fills
of a CAPTURED training step (bench.py --graph 1) that the eager step does not
have? Records one eager step and one (re)capture of the whole step under a
TorchDispatchMode (Python frames) and the CPU profiler (parent chains of the
ops the autograd threads run), and prints both tables.

    python tools/graph_op_sources.py --model gpt2
"""
import argparse
import os
import sys
import traceback
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = {"aten::copy_", "aten::add_", "aten::add", "aten::fill_", "aten::zero_", "aten::zeros", "aten::clone",
       "aten::_to_copy", "aten::cat", "aten::zeros_like", "aten::empty_like"}


def record(fn, pkg):
    from torch.profiler import ProfilerActivity, profile
    from torch.utils._python_dispatch import TorchDispatchMode

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

    chains = Counter()
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        with Spy():
            fn()
        torch.cuda.synchronize()
    for e in prof.events():
        if e.name not in OPS:
            continue
        names, p = [], e.cpu_parent
        while p is not None and len(names) < 4:
            names.append(p.name)
            p = p.cpu_parent
        chains[(e.name, " < ".join(names))] += 1
    return cnt, chains


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29000 + os.getpid() % 1000))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dev = torch.device("cuda", 0)
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd import workloads
    from distributed_compute_pytorch_amd.utils.graphs import capture_stream

    pkg = os.path.dirname(os.path.abspath(dcp.__file__))
    torch.manual_seed(0)
    wl = workloads.build(a.model, dev, fused=True)
    dcp.distributed.init_process_group("rccl", device_id=0)
    kw = {"defer_accum_wgrad": True} if wl.accum > 1 else {}
    with torch.cuda.stream(capture_stream()):
        ddp = dcp.parallel.DistributedDataParallel(wl.model, device_ids=[0], gradient_as_bucket_view=True,
                                                   **dcp.parallel.XGMI_BUCKETS, **kw)
        opt = wl.make_optimizer(ddp.parameters())
    eager = workloads.make_step(wl, ddp, opt)
    for _ in range(4):
        eager()
    torch.cuda.synchronize()
    ce, he = record(eager, pkg)
    graph_step = workloads.make_step(wl, ddp, opt, graph=True)  # eager warmup + capture
    graph_step()
    torch.cuda.synchronize()
    from distributed_compute_pytorch_amd.utils import graphs

    cap = [o for o in graph_step.__closure__ or [] if isinstance(o.cell_contents, graphs.CapturedStep)]
    captured = cap[0].cell_contents
    cg, hg = record(lambda: captured.recapture(warmup=0), pkg)
    keys = set(ce) | set(cg)
    print(f"# {a.model}: ATen ops (Python frame) per step: eager / captured")
    for k in sorted(keys, key=lambda k: -(cg.get(k, 0) - ce.get(k, 0))):
        if cg.get(k, 0) != ce.get(k, 0):
            print(f"{ce.get(k, 0):6d} {cg.get(k, 0):6d}  {k[0]:16s} {k[1]}")
    keys = set(he) | set(hg)
    print(f"# {a.model}: ATen ops (profiler parent chain) per step: eager / captured")
    for k in sorted(keys, key=lambda k: -(hg.get(k, 0) - he.get(k, 0)))[:a.top]:
        if hg.get(k, 0) != he.get(k, 0):
            print(f"{he.get(k, 0):6d} {hg.get(k, 0):6d}  {k[0]:16s} {k[1][:140]}")
    dcp.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
