"""Where does a training step's time go? Host vs device, per phase, ours vs torch.

python tools/step_breakdown.py --variant ours|torch|ours_ddp_torch_opt|torch_ddp_ours_opt [--model resnet50]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="ours")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--fused", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--profile", type=int, default=1)
    ap.add_argument("--fused-model", type=int, default=0, help="use fused kernels even with torch DDP")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29000 + os.getpid() % 1000))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd import workloads

    ours_ddp = a.variant in ("ours", "ours_ddp_torch_opt", "ours_nodpp_none")
    ours_opt = a.variant in ("ours", "torch_ddp_ours_opt")
    fused = bool(a.fused) and (ours_ddp or a.fused_model)
    wl = workloads.build(a.model, dev, batch=a.batch, fused=fused)
    if a.variant == "noddp_ours_opt":
        ddp = wl.model
        opt = wl.make_optimizer(ddp.parameters())
    elif ours_ddp:
        dcp.distributed.init_process_group("rccl", device_id=0)
        ddp = dcp.parallel.DistributedDataParallel(wl.model, device_ids=[0], gradient_as_bucket_view=True)
    else:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=dev)
        ddp = torch.nn.parallel.DistributedDataParallel(wl.model, device_ids=[0])
    if a.variant != "noddp_ours_opt":
        if ours_opt:
            opt = wl.make_optimizer(ddp.parameters())
        else:
            o = wl.make_optimizer([torch.nn.Parameter(torch.zeros(1, device=dev))])
            opt = getattr(torch.optim, type(o).__name__)(ddp.parameters(), **{
                k: v for k, v in o.defaults.items() if k != "decoupled_weight_decay"})
    step = workloads.make_step(wl, ddp, opt)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    # 1) free-running
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_host = (time.perf_counter() - t0) / a.steps
    torch.cuda.synchronize()
    t_total = (time.perf_counter() - t0) / a.steps
    # 2) phase-synchronised
    ph = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0}
    for _ in range(a.steps):
        b = next(wl.data)
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize(); t = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=wl.amp):
            loss = wl.loss_fn(ddp, b)
        torch.cuda.synchronize(); ph["fwd"] += time.perf_counter() - t; t = time.perf_counter()
        loss.backward()
        torch.cuda.synchronize(); ph["bwd"] += time.perf_counter() - t; t = time.perf_counter()
        opt.step()
        torch.cuda.synchronize(); ph["opt"] += time.perf_counter() - t
    res = {"variant": a.variant, "tag": a.tag, "fused": fused, "model": a.model, "free_running_ms": round(t_total * 1e3, 2),
           "host_issue_ms": round(t_host * 1e3, 2)}
    res.update({k + "_ms": round(v / a.steps * 1e3, 2) for k, v in ph.items()})
    print(json.dumps(res), flush=True)
    if a.profile:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                step()
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
