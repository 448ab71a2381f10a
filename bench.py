#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 DDP training throughput (samples/s, whole node).

BASELINE.json metric: "samples/sec (whole node) ResNet-50 DDP at 1/2/4/8
MI355X; scaling efficiency" on "ResNet-50 DDP bf16 ... synthetic ImageNet
224×224 batches". One process per GPU (torch.distributed.run or our
launcher), RCCL over xGMI, weak scaling (fixed per-GPU batch).

A step = zero_grad + forward (bf16 autocast, channels_last) + loss + backward
(bucketed RCCL all-reduce overlapped with backward) + fused optimizer update.
Synthetic data / random-init weights of the full-size model.

    python bench.py                                   # ResNet-50, 1 GPU
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8
    python bench.py --impl torch                      # stock torch DDP + torch.optim baseline
    python bench.py --model gpt2                      # GPT-2-small + grad accumulation (config #5)
    python bench.py --model bert                      # BERT-base pre-training (config #3)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

METRICS = {
    "resnet50": "samples/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X; scaling efficiency",
    "bert": "samples/sec (whole node) BERT-base DDP bf16",
    "gpt2": "samples/sec (whole node) GPT-2-small DDP + grad accumulation bf16",
    "convnet": "samples/sec (whole node) reference ConvNet DDP",
    "mlp": "samples/sec (whole node) 2-layer MLP DDP",
}


def _vs_baseline(model, wl, world, total):
    """value / (stock PyTorch DDP per-GPU throughput measured on MI355X x N):
    profiles/stock_baselines.json (BASELINE.md "Measured on MI355X"). None when
    the config differs from the measured one."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "stock_baselines.json")
    try:
        with open(path) as f:
            refs = json.load(f).get(model)
    except (OSError, ValueError):
        return None
    for ref in (refs if isinstance(refs, list) else [refs]):
        if ref and ref.get("per_gpu_batch") == wl.per_gpu_batch and ref.get("grad_accum", 1) == wl.accum \
                and ref.get("seq_len") == wl.seq_len:
            return round(total / (ref["samples_per_s_per_gpu"] * world), 4)
    return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50", choices=sorted(METRICS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU (micro-)batch")
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--accum", type=int, default=None, help="gradient-accumulation micro-steps")
    ap.add_argument("--impl", choices=["ours", "torch"], default="ours")
    ap.add_argument("--fused", "--fused-bn", dest="fused", type=int, default=1)
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--gemm", type=int, default=1, help="ResNet 1x1 convs as our MFMA GEMMs fused with BN")
    ap.add_argument("--bucket-cap-mb", type=float, default=None)
    ap.add_argument("--first-bucket-mb", type=float, default=None)
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--grad-as-view", type=int, default=1)
    ap.add_argument("--benchmark-cudnn", type=int, default=1)
    ap.add_argument("--graph", type=int, default=0, help="capture the whole step in a HIP graph")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def _heartbeat(period=30.0):
    """Print a progress line every `period` s from a daemon thread: the first
    steps on a fresh box (MIOpen kernel search / code-object loads) can run
    for minutes without the main thread printing anything."""
    import threading

    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            log(f"[bench] alive t={time.time() - t0:.0f}s")

    threading.Thread(target=run, daemon=True).start()


def main():
    a = parse()
    _heartbeat()
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
    from distributed_compute_pytorch_amd import workloads

    ours = a.impl == "ours"
    fused = bool(a.fused) and ours
    torch.manual_seed(0)
    wl = workloads.build(a.model, dev, batch=a.batch, fused=fused, seq_len=a.seq_len, accum=a.accum,
                         channels_last=bool(a.channels_last), fused_gemm=bool(a.gemm))

    import contextlib

    from distributed_compute_pytorch_amd.utils.graphs import capture_stream

    # graph capture: build DDP / optimizer under the capture stream (AccumulateGrad
    # nodes are bound to the stream current at their creation)
    stream_ctx = torch.cuda.stream(capture_stream()) if a.graph else contextlib.nullcontext()
    if ours:
        dcp.distributed.init_process_group("rccl", device_id=local)
        kw = {}
        if a.bucket_cap_mb is not None:
            kw["bucket_cap_mb"] = a.bucket_cap_mb
        if a.first_bucket_mb is not None:
            kw["first_bucket_mb"] = a.first_bucket_mb
        if a.comm_dtype == "bf16":
            kw["comm_dtype"] = torch.bfloat16
        with stream_ctx:
            ddp = dcp.parallel.DistributedDataParallel(wl.model, device_ids=[local],
                                                       gradient_as_bucket_view=bool(a.grad_as_view), **kw)
            opt = wl.make_optimizer(ddp.parameters())
        barrier = dcp.distributed.barrier

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
        with stream_ctx:
            ddp = torch.nn.parallel.DistributedDataParallel(wl.model, device_ids=[local], **kw)
        ours_opt = wl.make_optimizer([torch.nn.Parameter(torch.zeros(1, device=dev))])
        cls = getattr(torch.optim, type(ours_opt).__name__)
        opt = cls(ddp.parameters(), **{k: v for k, v in ours_opt.defaults.items()
                                       if k not in ("decoupled_weight_decay",)})
        barrier = tdist.barrier

        def max_over_ranks(x):
            t = torch.tensor([x], device=dev)
            tdist.all_reduce(t, tdist.ReduceOp.MAX)
            return float(t.item())

    step = workloads.make_step(wl, ddp, opt, graph=bool(a.graph))
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
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ms = elapsed / a.steps * 1000.0
    samples_per_step = wl.per_gpu_batch * wl.accum * world
    total = samples_per_step * a.steps / elapsed
    if rank == 0:
        cfg = {
            "model": a.model,
            "global_batch": samples_per_step,
            "per_gpu_batch": wl.per_gpu_batch,
            "grad_accum": wl.accum,
            "seq_len": wl.seq_len,
            "parallelism": f"dp{world}",
            "impl": a.impl,
            "fused_kernels": fused,
            "optimizer": type(opt).__name__,
            "comm_dtype": a.comm_dtype,
            "hip_graph": bool(a.graph),
        }
        if a.model == "resnet50":
            cfg["mfma_1x1_gemm"] = bool(a.gemm) and fused
        if a.model == "resnet50":
            cfg.update(image_size=224, channels_last=bool(a.channels_last))
        if ours:
            info = ddp.ddp_logging_data()
            cfg["buckets_mb"] = [round(b / 2**20, 2) for b in info["bucket_sizes"]]
        rec = {
            "metric": METRICS[a.model],
            "value": round(total, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if wl.amp else "fp32",
            "data": "synthetic (on-device random inputs/labels); random-init weights",
            "config": cfg,
        }
        if wl.seq_len:
            rec["tokens_per_s"] = round(total * wl.seq_len, 1)
        rec["vs_baseline"] = _vs_baseline(a.model, wl, world, total)
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if ours:
        dcp.distributed.destroy_process_group()
    else:
        import torch.distributed as tdist

        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
