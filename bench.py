#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 DDP training throughput (samples/s, whole node).

BASELINE.json metric: "samples/sec (whole node) ResNet-50 DDP at 1/2/4/8
MI355X; scaling efficiency" on "ResNet-50 DDP bf16 ... synthetic ImageNet
224×224 batches". One process per GPU (torch.distributed.run or our
launcher), RCCL over xGMI, weak scaling (fixed per-GPU batch).

A step = zero_grad + forward (bf16 autocast, channels_last) + cross-entropy +
backward (bucketed RCCL all-reduce overlapped) + fused SGD-momentum update.
Synthetic data / random-init weights of the full ResNet-50 (25.6 M params).

    python bench.py                       # 1 GPU, defaults
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 30 --warmup 10
    python bench.py --impl torch          # stock torch DDP + torch.optim.SGD baseline
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

BASELINE_METRIC = "samples/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X; scaling efficiency"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--impl", choices=["ours", "torch"], default="ours")
    ap.add_argument("--fused-bn", type=int, default=1)
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--bucket-cap-mb", type=float, default=None)
    ap.add_argument("--first-bucket-mb", type=float, default=None)
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--grad-as-view", type=int, default=1)
    ap.add_argument("--benchmark-cudnn", type=int, default=1)
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = bool(a.benchmark_cudnn)
    if "MASTER_ADDR" not in os.environ:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ.setdefault("MASTER_PORT", str(29400 + (os.getpid() % 1000)))
        os.environ["RANK"] = "0"
        os.environ["WORLD_SIZE"] = "1"

    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import resnet50

    fused_bn = bool(a.fused_bn) and a.impl == "ours"
    torch.manual_seed(0)
    model = resnet50(fused_bn=fused_bn).to(dev)
    if a.channels_last:
        model = model.to(memory_format=torch.channels_last)

    if a.impl == "ours":
        dcp.distributed.init_process_group("rccl", device_id=local)
        kw = {}
        if a.bucket_cap_mb is not None:
            kw["bucket_cap_mb"] = a.bucket_cap_mb
        if a.first_bucket_mb is not None:
            kw["first_bucket_mb"] = a.first_bucket_mb
        if a.comm_dtype == "bf16":
            kw["comm_dtype"] = torch.bfloat16
        ddp = dcp.parallel.DistributedDataParallel(model, device_ids=[local], gradient_as_bucket_view=bool(
            a.grad_as_view), **kw)
        opt = dcp.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        barrier = lambda: dcp.distributed.barrier()  # noqa: E731

        def max_over_ranks(x):
            t = torch.tensor([x], device=dev)
            dcp.distributed.all_reduce(t, dcp.distributed.ReduceOp.MAX)
            return float(t.item())
    else:
        import torch.distributed as tdist

        tdist.init_process_group("nccl", device_id=dev)
        kw = {}
        if a.bucket_cap_mb is not None:
            kw["bucket_cap_mb"] = a.bucket_cap_mb
        ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], **kw)
        opt = torch.optim.SGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        barrier = lambda: tdist.barrier()  # noqa: E731

        def max_over_ranks(x):
            t = torch.tensor([x], device=dev)
            tdist.all_reduce(t, tdist.ReduceOp.MAX)
            return float(t.item())

    data = dcp.utils.SyntheticBatches(a.batch, (3, 224, 224), 1000, dev, channels_last=bool(a.channels_last),
                                      pool=2)

    def step():
        x, y = next(data)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = ddp(x)
            loss = F.cross_entropy(out, y)
        loss.backward()
        opt.step()
        return loss

    t_w = time.time()
    for i in range(a.warmup):
        loss = step()
        if rank == 0 and (i == 0 or (i + 1) % 5 == 0):
            torch.cuda.synchronize()
            log(f"[bench] warmup {i + 1}/{a.warmup} loss={loss.item():.4f} t={time.time() - t_w:.1f}s")
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed)
    ms = elapsed / a.steps * 1000.0
    total = a.batch * world * a.steps / elapsed
    if rank == 0:
        rec = {
            "metric": BASELINE_METRIC,
            "value": round(total, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (on-device random 224x224 images, random labels); random-init weights",
            "config": {
                "model": "resnet50",
                "global_batch": a.batch * world,
                "per_gpu_batch": a.batch,
                "seq_len": None,
                "image_size": 224,
                "parallelism": f"dp{world}",
                "impl": a.impl,
                "fused_bn": fused_bn,
                "channels_last": bool(a.channels_last),
                "optimizer": "SGD(momentum=0.9, wd=1e-4)",
                "comm_dtype": a.comm_dtype,
            },
        }
        if a.impl == "ours":
            info = ddp.ddp_logging_data()
            rec["config"]["buckets_mb"] = [round(b / 2**20, 2) for b in info["bucket_sizes"]]
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if a.impl == "ours":
        dcp.distributed.destroy_process_group()
    else:
        import torch.distributed as tdist

        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
