"""Multi-process GPU test helper: N ranks, rank r on device r % ndev.

``backend="rccl"`` needs one GPU per rank (RCCL refuses two ranks on one
device); ``backend="gloo"`` (our host communicator staging device tensors,
the reference-literal mode of main.py:50) can put several ranks on one GPU.
Each rank also gets a stock torch.distributed group (``torch_backend``) on a
second port so tests can run ``torch.nn.parallel.DistributedDataParallel``
side by side with ours.
"""
import datetime
import os

from distributed_compute_pytorch_amd.distributed.launch import free_port, spawn


def _entry(rank, fn, world, port, backend, torch_backend, pg_timeout_s, args, port2=None):
    import torch

    ndev = torch.cuda.device_count()
    dev = rank % ndev
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(dev))
    import distributed_compute_pytorch_amd as dcp

    dcp.distributed.init_process_group(backend, device_id=dev if backend in ("rccl", "nccl") else None,
                                       timeout=datetime.timedelta(seconds=pg_timeout_s))
    tdist = None
    if torch_backend:
        import torch.distributed as tdist

        kw = {"device_id": torch.device("cuda", dev)} if torch_backend == "nccl" else {}
        tdist.init_process_group(torch_backend, init_method=f"tcp://127.0.0.1:{port2 or port + 1}", rank=rank,
                                 world_size=world, timeout=datetime.timedelta(seconds=120), **kw)
    try:
        fn(rank, world, torch.device("cuda", dev), *args)
    finally:
        if tdist is not None:
            tdist.destroy_process_group()
        dcp.distributed.destroy_process_group()


def run_gpu_world(fn, world, *args, backend="rccl", torch_backend=None, timeout=240, pg_timeout_s=120.0):
    port = free_port()
    port2 = free_port()  # the stock torch group's own free port (port + 1 may be taken)
    while port2 == port:
        port2 = free_port()
    spawn(_entry, (fn, world, port, backend, torch_backend, pg_timeout_s, args, port2), nprocs=world,
          timeout=timeout)
