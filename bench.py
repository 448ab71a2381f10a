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
    python bench.py --gpus 8                          # self-launches 8 ranks (parent never touches a GPU)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8         # same, under torchrun (the driver's form)
    python bench.py --comm-timing 1                   # + per-bucket ready/comm ms, exposed comm ms
    python bench.py --bucket-sweep 4,8,16,25,50,100   # config #4: one JSON line per bucket cap (MiB)
    python bench.py --gpus 8 --ref-1gpu 11200         # + scaling_efficiency vs a 1-GPU samples/s
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
    ap.add_argument("--tail-bucket-mb", type=float, default=None,
                    help="size of the ready-last tail bucket split off the plan (0 = no split)")
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--overlap-optimizer", type=int, default=-1,
                    help="DDP overlap_optimizer: the fused optimizer updates each bucket's parameters as soon as "
                         "its reduction lands (-1: on for the transformers, whose ready-last embedding bucket "
                         "is 90-150 MB)")
    ap.add_argument("--grad-as-view", type=int, default=1)
    ap.add_argument("--defer-wgrad", type=int, default=-1,
                    help="DDP defer_accum_wgrad: the no_sync micro-steps' Linear weight gradients are computed by the "
                         "synchronising micro-step in one launch over all micro-steps' rows (-1: on when grad_accum > 1)")
    ap.add_argument("--benchmark-cudnn", type=int, default=1)
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the whole step in a HIP graph (-1: per model — on for the launch-bound "
                         "reference ConvNet / MLP and for the transformers at one rank, off otherwise)")
    ap.add_argument("--backend", choices=["rccl", "gloo"], default="rccl",
                    help="gloo: the reference's literal backend (main.py:50) — GPU tensors staged through the "
                         "host; ours = the C++ host communicator, stock = torch's gloo")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--comm-timing", type=int, default=0,
                    help="record per-bucket device comm time + exposed (un-overlapped) comm ms in the JSON")
    ap.add_argument("--bucket-sweep", default=None,
                    help="comma-separated bucket caps in MiB: one timed run and one JSON line per cap")
    ap.add_argument("--ref-1gpu", type=float, default=None,
                    help="1-GPU samples/s of the same config: adds scaling_efficiency = value / (N * ref)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="1 GPU only: every bucket all-reduce is replaced by a contention emulation of an N-rank "
                         "ring all-reduce on the comm stream (parallel/comm_hooks.py; NOTES §22)")
    ap.add_argument("--emulate-busbw", type=float, default=300.0, help="emulated bus bandwidth, GB/s")
    ap.add_argument("--emulate-channels", type=int, default=16, help="emulated RCCL channels (workgroups)")
    ap.add_argument("--reserve-cus", type=int, default=None,
                    help="CUs the persistent GEMM / conv grids leave free for collectives (DCP_RESERVE_CUS)")
    ap.add_argument("--linear-path", choices=["ours", "ours-unfused-mlp", "aten-fwd", "aten"], default="ours",
                    help="transformer Linear forward / data-gradient GEMMs: ours (gemm_nt + fused epilogues), "
                         "aten-fwd (forward on hipBLASLt), aten (forward and dgrad on hipBLASLt)")
    ap.add_argument("--pro-max-cout", type=int, default=None,
                    help="ResNet: BN2 + ReLU as conv3's GEMM prologue while Cout <= this (models/resnet.py PRO_MAX_COUT)")
    ap.add_argument("--res-prologue", type=int, default=0,
                    help="ResNet identity block boundaries: BN3 + residual + ReLU as the next conv1's GEMM prologue "
                         "(1; default 0 = separate apply pass, measured faster: ops/conv.py RES_PROLOGUE)")
    ap.add_argument("--grad-to-none", type=int, default=1,
                    help="zero_grad(set_to_none=...) in the step: 1 (torch's default, as main.py) or 0 (zero in place)")
    ap.add_argument("--gemm-tune", default=None,
                    help="k=v[,k=v] entries of the GEMM launcher tuning table (_C.gemm_tune, e.g. nt_big=4)")
    return ap.parse_args()


def _visible_gpus() -> int:
    """GPUs this process could use, counted WITHOUT the HIP runtime (the
    self-launching parent must not create a device context): the KFD topology
    nodes with a non-zero gpu_id, narrowed by a *_VISIBLE_DEVICES list."""
    import glob

    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            with open(f) as fh:
                n += int(fh.read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([d for d in v.split(",") if d.strip() != ""]))
    return n


def _self_launch(a) -> int:
    """``--gpus N`` without a launcher: start N ranks of this script (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set, one process per GPU) and return the
    job's exit code; rank 0 prints the JSON line. The parent never touches the
    HIP runtime (it counts GPUs from sysfs) and does not import the package
    (its extension links the HIP runtime)."""
    import importlib.util

    n = _visible_gpus()
    if n < a.gpus and a.backend != "gloo":
        log(f"[bench] --gpus {a.gpus} requested but only {n} GPU(s) are visible; refusing to oversubscribe "
            f"(RCCL needs one device per rank)")
        return 2
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location(
        "_dcp_launch", os.path.join(here, "distributed_compute_pytorch_amd", "distributed", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    log(f"[bench] self-launching {a.gpus} ranks")
    return mod.launch_env([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], a.gpus,
                          master_addr="127.0.0.1")


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
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # decided before ANY torch.cuda call: the parent must not own a GPU context
        raise SystemExit(_self_launch(a))
    _heartbeat()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.graph < 0:
        # the launch-bound reference ConvNet / MLP, and the transformers at one
        # rank: their eager step idles the GPU between dependent kernels on a
        # slow host (BERT 0.915 busy; captured 0.995, +4.6 % on such a box,
        # parity on a fast one: profiles/r6_graph_ab*.jsonl, NOTES §31). At
        # N > 1 the transformers run eager (optimizer overlap with the
        # bucket collectives)
        a.graph = 1 if (a.impl == "ours" and a.backend == "rccl"
                        and (a.model in ("convnet", "mlp") or (a.model in ("gpt2", "bert") and world == 1))) else 0
    if world != a.gpus:
        log(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if a.comm_timing:
        os.environ["DCP_COMM_TIMING"] = "1"  # read by the communicator / Reducer at construction
    if a.emulate_world:
        if world != 1:
            raise SystemExit("--emulate-world stands in for the peers of a 1-GPU run")
        os.environ["DCP_SINGLE_RANK_HOP"] = "1"  # collectives on the comm stream, as at N > 1
    if a.reserve_cus is not None:
        os.environ["DCP_RESERVE_CUS"] = str(a.reserve_cus)  # read when the extension loads
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if a.backend == "gloo":
        # host-staged collectives: ranks may share a GPU (reference-literal runs on a small box)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = bool(a.benchmark_cudnn)
    if "WORLD_SIZE" not in os.environ:  # a plain single-process run
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29400 + (os.getpid() % 1000)))
        os.environ["RANK"] = "0"
        os.environ["WORLD_SIZE"] = "1"

    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd import workloads

    ours = a.impl == "ours"
    fused = bool(a.fused) and ours
    tune = {}
    if a.gemm_tune:
        from distributed_compute_pytorch_amd._ext import C as _C

        for kv in a.gemm_tune.split(","):
            k, v = kv.split("=")
            _C.gemm_tune(k.strip(), int(v))
            tune[k.strip()] = _C.gemm_tune_get(k.strip())
    if a.pro_max_cout is not None:
        from distributed_compute_pytorch_amd.models import resnet as _resnet

        _resnet.PRO_MAX_COUT = a.pro_max_cout
    if a.res_prologue:
        from distributed_compute_pytorch_amd.ops import conv as _conv_ops

        _conv_ops.RES_PROLOGUE = True
    if a.linear_path != "ours":
        from distributed_compute_pytorch_amd.ops import linear as _lin

        _lin._FUSED_MLP = False
        if a.linear_path != "ours-unfused-mlp":
            _lin._OUR_FWD = False
            _lin._OUR_DGRAD = a.linear_path == "aten-fwd"
    torch.manual_seed(0)
    wl = workloads.build(a.model, dev, batch=a.batch, fused=fused, seq_len=a.seq_len, accum=a.accum,
                         channels_last=bool(a.channels_last), fused_gemm=bool(a.gemm))

    import contextlib

    from distributed_compute_pytorch_amd.utils.graphs import capture_stream

    # graph capture: build DDP / optimizer under the capture stream (AccumulateGrad
    # nodes are bound to the stream current at their creation)
    stream_ctx = (lambda: torch.cuda.stream(capture_stream())) if a.graph else contextlib.nullcontext
    if ours:
        dcp.distributed.init_process_group(a.backend, device_id=local if a.backend == "rccl" else None)
        barrier = dcp.distributed.barrier
        all_reduce, MAX = dcp.distributed.all_reduce, dcp.distributed.ReduceOp.MAX
    else:
        import torch.distributed as tdist

        if a.backend == "gloo":
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=dev)
        barrier = tdist.barrier
        all_reduce, MAX = tdist.all_reduce, tdist.ReduceOp.MAX

    def max_over_ranks(x):
        t = torch.tensor([x], device=dev)
        all_reduce(t, MAX)
        return float(t.item())

    def build_ddp(cap_mb):
        kw = {}
        if cap_mb is not None:
            kw["bucket_cap_mb"] = cap_mb
        if ours:
            # the xGMI-tuned bucket plan (NOTES §18) unless overridden on the CLI
            kw = {**dcp.parallel.XGMI_BUCKETS, **kw}
            if a.first_bucket_mb is not None:
                kw["first_bucket_mb"] = a.first_bucket_mb
            if a.tail_bucket_mb is not None:
                kw["tail_bucket_mb"] = a.tail_bucket_mb
            if a.comm_dtype == "bf16":
                kw["comm_dtype"] = torch.bfloat16
            # optimizer / all-reduce overlap: only with collectives to overlap
            # (one rank: the chunked step is pure host overhead, NOTES §28)
            ov = a.overlap_optimizer if a.overlap_optimizer >= 0 else int(a.model in ("gpt2", "bert") and world > 1)
            if ov and a.grad_as_view:
                kw["overlap_optimizer"] = True
            if (a.defer_wgrad if a.defer_wgrad >= 0 else int(wl.accum > 1)):
                kw["defer_accum_wgrad"] = True
            with stream_ctx():
                ddp = dcp.parallel.DistributedDataParallel(wl.model, device_ids=[local],
                                                           gradient_as_bucket_view=bool(a.grad_as_view), **kw)
                opt = wl.make_optimizer(ddp.parameters())
            if a.emulate_world:
                from distributed_compute_pytorch_amd.parallel import comm_hooks

                ddp.register_comm_hook(comm_hooks.ContentionEmulation(a.emulate_world, a.emulate_busbw,
                                                                      a.emulate_channels),
                                       comm_hooks.contention_emulation_hook)
            return ddp, opt
        with stream_ctx():
            ddp = torch.nn.parallel.DistributedDataParallel(wl.model, device_ids=[local], **kw)
        ours_opt = wl.make_optimizer([torch.nn.Parameter(torch.zeros(1, device=dev))])
        cls = getattr(torch.optim, type(ours_opt).__name__)
        opt = cls(ddp.parameters(), **{k: v for k, v in ours_opt.defaults.items()
                                       if k not in ("decoupled_weight_decay",)})
        return ddp, opt

    def timed_run(cap_mb):
        ddp, opt = build_ddp(cap_mb)
        if ours and world > 1 and workloads.pretune_step(wl, ddp, opt):
            # GEMM autotune outside any synchronised backward (no bucket
            # collective in flight), one rank-0 table for all ranks
            log(f"[bench] rank {rank}: GEMM shapes tuned in a no_sync micro-step")
        step = workloads.make_step(wl, ddp, opt, graph=bool(a.graph), set_to_none=bool(a.grad_to_none))
        t_w = time.time()
        for i in range(a.warmup):
            loss = step()
            if rank == 0 and (i == 0 or (i + 1) % 5 == 0):
                torch.cuda.synchronize()
                log(f"[bench] warmup {i + 1}/{a.warmup} loss={loss.item():.4f} t={time.time() - t_w:.1f}s")
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        prof = None
        if os.environ.get("DCP_BENCH_CPROFILE"):  # host-side profile of the timed steps only (diagnostics)
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        for i in range(a.steps):
            loss = step()
        t_host = time.perf_counter() - t0  # host time to enqueue the steps (the GPU may still be running)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        elapsed = max_over_ranks(time.perf_counter() - t0)
        if prof is not None:
            prof.disable()
            prof.dump_stats(os.environ["DCP_BENCH_CPROFILE"])
            log(f"[bench] host enqueue time {t_host / a.steps * 1e3:.2f} ms/step vs {elapsed / a.steps * 1e3:.2f} ms/step")
        ms = elapsed / a.steps * 1000.0
        samples_per_step = wl.per_gpu_batch * wl.accum * world
        total = samples_per_step * a.steps / elapsed
        rec = None
        diag = None
        if ours and (world > 1 or a.emulate_world) and not a.comm_timing and not a.graph:
            # untimed diagnostic steps with device comm timing on: whether
            # overlap held (exposed vs per-bucket comm ms), as a multi-GPU run
            # record must be able to explain itself; MAX over ranks
            ddp.set_comm_timing(True)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            info = ddp.ddp_logging_data()
            ddp.set_comm_timing(False)
            diag = {
                "steps": 3,
                "exposed_comm_ms": round(max_over_ranks(info["exposed_comm_ms"]), 4),
                "bucket_comm_ms": [round(x, 4) for x in info["bucket_comm_ms"]],
                "bucket_ready_dev_ms": [round(x, 3) for x in info["bucket_ready_dev_ms"]],
                "comm_bytes_per_step": sum(info["bucket_sizes"]),
                "rccl_ranks": ddp._comm.transport_size(),
                "backend": info["backend"],
            }
        if ours:
            info = ddp.ddp_logging_data()
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
                "grad_to_none": bool(a.grad_to_none),
                "backend": a.backend,
            }
            if a.model == "resnet50":
                cfg.update(mfma_1x1_gemm=bool(a.gemm) and fused, image_size=224, channels_last=bool(a.channels_last),
                           res_prologue=bool(a.res_prologue) and fused)
                if a.pro_max_cout is not None:
                    cfg["pro_max_cout"] = a.pro_max_cout
            if a.emulate_world:
                cfg["emulated_comm"] = {"world": a.emulate_world, "busbw_gbps": a.emulate_busbw,
                                        "channels": a.emulate_channels}
            if a.reserve_cus is not None:
                cfg["reserve_cus"] = a.reserve_cus
            if tune:
                cfg["gemm_tune"] = tune
            if a.linear_path != "ours":
                cfg["linear_path"] = a.linear_path
            if a.model in ("gpt2", "bert") and ours:
                from distributed_compute_pytorch_amd.ops.linear import autotune_choices, autotune_times

                cfg["linear_gemm_choice"] = autotune_choices()
                cfg["linear_gemm_us_by_candidate"] = autotune_times()
            if ours:
                cfg["bucket_cap_mb"] = round(info["bucket_cap_bytes"] / 2**20, 3)
                cfg["first_bucket_mb"] = round(info["first_bucket_bytes"] / 2**20, 3)
                cfg["tail_bucket_mb"] = round(ddp.tail_bucket_bytes / 2**20, 3)
                cfg["overlap_optimizer"] = bool(ddp.overlap_optimizer)
                cfg["defer_accum_wgrad"] = bool(getattr(ddp, "defer_accum_wgrad", False))
                cfg["buckets_mb"] = [round(b / 2**20, 2) for b in info["bucket_sizes"]]
            elif cap_mb is not None:
                cfg["bucket_cap_mb"] = cap_mb
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
            rec["peak_mem_gib"] = round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
            rec["vs_baseline"] = _vs_baseline(a.model, wl, world, total)
            if diag is not None:
                rec["comm_diag"] = diag
            if a.ref_1gpu:
                rec["scaling_efficiency"] = round(total / (world * a.ref_1gpu), 4)
            if ours and a.comm_timing:
                # last timed iteration: when each bucket became ready (host ms
                # since backward start), its collective's device time, and the
                # device time the step waited for communication after backward
                rec["comm"] = {
                    "bucket_ready_ms": [round(x, 3) for x in info["bucket_ready_ms"]],
                    "bucket_ready_dev_ms": [round(x, 3) for x in info["bucket_ready_dev_ms"]],
                    "bucket_comm_ms": [round(x, 4) for x in info["bucket_comm_ms"]],
                    "exposed_comm_ms": round(info["exposed_comm_ms"], 4),
                    "comm_bytes_per_step": sum(info["bucket_sizes"]),
                }
        del step, ddp, opt
        return rec

    caps = [float(c) for c in a.bucket_sweep.split(",")] if a.bucket_sweep else [a.bucket_cap_mb]
    for cap in caps:
        rec = timed_run(cap)
        if rec is not None:
            line = json.dumps(rec)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "a" if a.bucket_sweep else "w") as f:
                    f.write(line + "\n")
        import gc

        gc.collect()
    if ours:
        dcp.distributed.destroy_process_group()
    else:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
