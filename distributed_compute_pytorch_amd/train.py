"""General trainer CLI: the reference's proc()/train()/test() loop (main.py:55-134)
on this framework, for every model family, with structured metrics,
checkpoint/resume, optional whole-step HIP-graph capture (``--hip-graph``)
and a torch.profiler trace of the first epoch (``--profile``).

    python -m distributed_compute_pytorch_amd.train --model convnet --gpus 2 --epochs 1
    python -m distributed_compute_pytorch_amd.distributed.run --nproc-per-node 8 \
        -m distributed_compute_pytorch_amd.train --model resnet50 --dtype bf16 --steps-per-epoch 100

Launched without RANK in the environment it spawns ``--gpus`` ranks itself
(like the reference's mp.spawn, main.py:150); under a launcher it runs as the
given rank.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

from . import distributed as dist
from .config import TrainConfig, parse_config


def _device(cfg: TrainConfig, local_rank: int):
    if not cfg.no_cuda and torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
        return torch.device("cuda", local_rank)
    return torch.device("cpu")


def _mnist_loaders(cfg, rank, world):
    from .utils.data import DistributedSampler, MNISTIdx, SyntheticDataset

    try:
        if cfg.synthetic:
            raise FileNotFoundError
        tr, te = MNISTIdx(cfg.data_dir, True), MNISTIdx(cfg.data_dir, False)
    except FileNotFoundError:
        tr, te = SyntheticDataset(60000, seed=cfg.seed), SyntheticDataset(10000, seed=cfg.seed + 1)
    s_tr = DistributedSampler(tr, world, rank, seed=cfg.seed)
    s_te = DistributedSampler(te, world, rank, shuffle=False)
    pin = not cfg.no_cuda and torch.cuda.is_available()
    return (DataLoader(tr, batch_size=cfg.batch_size, sampler=s_tr, pin_memory=pin), s_tr,
            DataLoader(te, batch_size=cfg.batch_size, sampler=s_te, pin_memory=pin))


def run_rank(cfg: TrainConfig, rank: int, world: int, local_rank: int):
    from . import ops
    from . import workloads
    from .parallel import DistributedDataParallel
    from .utils import JsonLogger, load_checkpoint, save_checkpoint, save_model

    device = _device(cfg, local_rank)
    backend = cfg.backend if cfg.backend != "auto" else ("rccl" if device.type == "cuda" else "host")
    if not dist.is_initialized():
        dist.init_process_group(backend, rank=rank, world_size=world,
                                device_id=local_rank if device.type == "cuda" else None)
    torch.manual_seed(cfg.seed)
    log = JsonLogger(rank, cfg.metrics_file, stream=sys.stdout)
    mnist = cfg.model in ("convnet", "mlp")
    wl = workloads.build(cfg.model, device, batch=cfg.batch_size, fused=device.type == "cuda",
                         accum=cfg.grad_accum, channels_last=device.type == "cuda")
    if mnist:
        wl.amp = cfg.dtype == "bf16"
    from .parallel import XGMI_BUCKETS

    kw = dict(XGMI_BUCKETS)  # xGMI-tuned bucket plan (NOTES §18); the CLI overrides it
    if cfg.bucket_cap_mb:
        kw["bucket_cap_mb"] = cfg.bucket_cap_mb
    if cfg.first_bucket_mb:
        kw["first_bucket_mb"] = cfg.first_bucket_mb
    if cfg.comm_dtype == "bf16":
        kw["comm_dtype"] = torch.bfloat16
    # --hip-graph: the DDP model, the optimizer and every training step (eager
    # warmups, capture, replays) live on ONE side stream — torch refuses to
    # capture the default stream, and the autograd engine binds each
    # parameter's AccumulateGrad node (which the Reducer hooks) to the stream
    # current when it was created (utils/graphs.py)
    graph = bool(cfg.hip_graph) and device.type == "cuda"
    if graph:
        from .utils.graphs import capture_stream

        side = capture_stream(device.index)
        side.wait_stream(torch.cuda.current_stream())

        def step_ctx():
            return torch.cuda.stream(side)
    else:
        side = None
        step_ctx = _Null
    with step_ctx():
        model = DistributedDataParallel(wl.model, device_ids=[local_rank] if device.type == "cuda" else None,
                                        broadcast_buffers=cfg.broadcast_buffers,
                                        find_unused_parameters=cfg.find_unused_parameters,
                                        gradient_as_bucket_view=cfg.gradient_as_bucket_view, **kw)
        opt = wl.make_optimizer(model.parameters())
    for g in opt.param_groups:
        g["lr"] = cfg.lr if mnist else g["lr"]
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=cfg.gamma)
    start_epoch = 0
    if cfg.resume and os.path.exists(cfg.resume):
        meta = load_checkpoint(cfg.resume, model, opt, sched, map_location=device)
        start_epoch = meta["epoch"] + 1
        log.log(event="resumed", epoch=meta["epoch"])
    log.log(event="config", rank0_device=str(device), world_size=world, config=cfg.to_json())

    if mnist:
        train_loader, train_sampler, test_loader = _mnist_loaders(cfg, rank, world)
    step = None
    losslog = _LossLog(log)
    for epoch in range(start_epoch, cfg.epochs):
        model.train()
        t0 = time.time()
        seen = 0
        if mnist:
            train_sampler.set_epoch(epoch)
            batches = iter(train_loader)
            nsteps = len(train_loader) if not cfg.steps_per_epoch else min(cfg.steps_per_epoch, len(train_loader))
        else:
            batches = wl.data
            nsteps = cfg.steps_per_epoch or 100
        prof = _profiler(cfg, rank, epoch == start_epoch)
        for b in range(nsteps):
            with step_ctx():  # H2D copies, the step and the loss logging in one stream order
                flat = []
                for _k in range(wl.accum):
                    bt = tuple(t.to(device, non_blocking=True) for t in next(batches))
                    seen += bt[0].shape[0]
                    flat.extend(bt)
                if step is None:
                    step = _make_step(cfg, wl, model, opt, device, side)
                loss = step(*flat)
                if prof is not None:
                    prof.step()
                if b % cfg.log_every == 0:
                    t = loss.detach().float().clone() * wl.accum
                    dist.all_reduce(t, dist.ReduceOp.AVG if t.is_cuda else dist.ReduceOp.SUM)
                    if not t.is_cuda:
                        t /= world
                    losslog.push(t, epoch=epoch, step=b, steps=nsteps, lr=opt.param_groups[0]["lr"])
                losslog.poll()
        losslog.poll(wait=True)
        if prof is not None:
            prof.stop()
            path = (cfg.metrics_file or "dcp") + f".trace.rank{rank}.json"
            prof.export_chrome_trace(path)
            log.log(event="profile", trace=path)
        if device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.time() - t0
        log.log(event="epoch", epoch=epoch, seconds=round(dt, 3),
                samples_per_s=round(seen * world / max(dt, 1e-9), 1))
        if mnist:
            model.eval()
            m = ops.EvalMetrics(device, log_probs=True)
            with torch.no_grad():
                for img, label in test_loader:
                    m.update(model(img.to(device)), label.to(device))
            avg, acc, n = m.compute()
            log.log(event="eval", epoch=epoch, avg_loss=round(avg, 6), accuracy=round(acc, 6), samples=n)
        sched.step()
        if cfg.checkpoint:
            save_checkpoint(cfg.checkpoint, model, opt, sched, epoch=epoch)
    if cfg.save_model:
        save_model(model, cfg.save_model)
    dist.destroy_process_group()


class _LossLog:
    """The logged training loss without a host stall. The reference reads
    ``loss.item()`` right after its all-reduce (``main.py:65-68``), which
    drains the GPU queue at every logged step. Here the averaged loss is
    copied into pinned host memory behind an event on the step's stream (so
    a replayed graph's static output is read before the next replay) and the
    record is written once the event has completed: polled every step,
    flushed at the end of the epoch, in step order."""

    def __init__(self, log):
        self.log = log
        self.q = []

    def push(self, t: torch.Tensor, **fields):
        if not t.is_cuda:
            self._write(t.item(), fields)
            return
        h = torch.empty((), dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.q.append((h, ev, fields))

    def poll(self, wait: bool = False):
        while self.q and (wait or self.q[0][1].query()):
            h, ev, fields = self.q.pop(0)
            ev.synchronize()
            self._write(h.item(), fields)

    def _write(self, v: float, f: dict):
        self.log.log(event="train", epoch=f["epoch"], step=f["step"], steps=f["steps"], loss=round(v, 6),
                     lr=f["lr"])


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _make_step(cfg: TrainConfig, wl, model, opt, device, side=None):
    """One optimizer step over ``wl.accum`` micro-batches (all but the last
    under ``no_sync``; backward runs INSIDE the context, like the forward).
    ``cfg.hip_graph`` on a GPU: the whole step (forward, backward, bucket
    reduction, clipping, optimizer) is captured once and replayed."""

    def run(*flat):
        opt.zero_grad(set_to_none=True)
        n = len(flat) // wl.accum
        loss = None
        for k in range(wl.accum):
            bt = flat[k * n:(k + 1) * n]
            ctx = model.no_sync() if k < wl.accum - 1 else _Null()
            with ctx:
                with torch.autocast(device.type, dtype=torch.bfloat16, enabled=wl.amp):
                    loss = wl.loss_fn(model, bt) / wl.accum
                loss.backward()
        if cfg.clip_grad_norm > 0:
            from .optim import clip_grad_norm_
            clip_grad_norm_(model.parameters(), cfg.clip_grad_norm)
        opt.step()
        return loss

    if not (cfg.hip_graph and device.type == "cuda"):
        return run
    from .utils.graphs import CapturedStep

    for g in opt.param_groups:
        if "capturable" in g:
            g["capturable"] = True
    # the DDP model was built on the side stream (run_rank); capture on it too
    # (the Reducer's AccumulateGrad nodes are bound to their creation stream).
    # The first two steps run eagerly on real batches (bucket rebuild,
    # optimizer state, kernel tables); the third is captured (capture executes
    # nothing) and replayed: no extra training steps on a static batch. One
    # graph memory pool serves every (re)capture.
    st = {"eager": 0, "cap": None, "lr": None, "recaptures": 0, "calls": 0}

    def call(*flat):
        lrs = [g["lr"] for g in opt.param_groups]
        if st["cap"] is None:
            if st["eager"] < 2:
                st["eager"] += 1
                return run(*flat)
            st["cap"] = CapturedStep(run, [t.clone() for t in flat], warmup=0, stream=side,
                                     pool=torch.cuda.graph_pool_handle())
            st["lr"] = lrs
        cap = st["cap"]
        st["calls"] += 1
        if lrs != st["lr"]:  # the captured kernels hold the LR as a constant
            st["lr"] = lrs
            st["recaptures"] += 1
            if st["recaptures"] > 2 and st["calls"] < 20 * st["recaptures"]:
                import warnings

                warnings.warn("--hip-graph: the learning rate changes almost every step, so the step is "
                              "re-captured each time (slower than eager); use a per-epoch schedule",
                              stacklevel=2)
            cap.recapture(warmup=0)
        if all(a.shape == b.shape for a, b in zip(flat, cap.static_inputs)):
            return cap(*flat)
        return run(*flat)  # ragged last batch of an epoch: eager

    return call


def _profiler(cfg: TrainConfig, rank: int, first_epoch: bool):
    """``cfg.profile``: torch.profiler over steps 2-6 of the first epoch (CPU +
    HIP activity, our roctx/record_function ranges included); the chrome trace
    lands next to the metrics file."""
    if not (cfg.profile and first_epoch):
        return None
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available() and not cfg.no_cuda:
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    p = torch.profiler.profile(activities=acts, schedule=torch.profiler.schedule(wait=1, warmup=1, active=5,
                                                                                 repeat=1))
    p.start()
    return p


def _spawn_entry(rank, cfg, world, port):
    os.environ.update(MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port))
    run_rank(cfg, rank, world, rank)


def main(argv=None):
    cfg = parse_config(argv)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        run_rank(cfg, int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]),
                 int(os.environ.get("LOCAL_RANK", os.environ["RANK"])))
        return
    world = cfg.gpus
    if not cfg.no_cuda and torch.cuda.is_available() and world > torch.cuda.device_count():
        raise SystemExit(f"--gpus {world} but only {torch.cuda.device_count()} GPUs are visible")
    from .distributed.launch import free_port, spawn

    spawn(_spawn_entry, (cfg, world, int(os.environ.get("MASTER_PORT", free_port()))), nprocs=world)


if __name__ == "__main__":
    main()
