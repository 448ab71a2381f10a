"""Helpers for multi-process CPU tests (host backend, 127.0.0.1 rendezvous)."""
import os

from distributed_compute_pytorch_amd.distributed.launch import free_port, spawn


def _entry(rank, fn, world, port, backend, args, port2=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    if port2 is not None:  # a second free port for a stock torch.distributed twin group
        os.environ["DCP_TEST_TORCH_PORT"] = str(port2)
    import distributed_compute_pytorch_amd as dcp

    if backend is not None:
        dcp.distributed.init_process_group(backend)
    try:
        fn(rank, world, *args)
    finally:
        if backend is not None:
            dcp.distributed.destroy_process_group()


def run_world(fn, world=2, *args, backend="gloo", timeout=180):
    port = free_port()
    port2 = free_port()
    while port2 == port:
        port2 = free_port()
    spawn(_entry, (fn, world, port, backend, args, port2), nprocs=world, timeout=timeout)
