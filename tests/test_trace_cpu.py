"""Tracing ranges (roctx + torch profiler) and DDP observability fields."""
import torch

from distributed_compute_pytorch_amd.utils.trace import mark, roctx_available, trace_range


def test_trace_range_visible_in_torch_profiler():
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        with trace_range("dcp.test.region"):
            torch.ones(4).sum()
        mark("dcp.test.mark")
    names = {e.name for e in prof.events()}
    assert "dcp.test.region" in names
    assert isinstance(roctx_available(), bool)


def test_ddp_forward_range_and_logging(tmp_path):
    from mp_util import run_world

    run_world(_ddp_worker, 1)


def _ddp_worker(rank, world):
    import distributed_compute_pytorch_amd as dcp

    m = torch.nn.Linear(8, 4)
    ddp = dcp.parallel.DistributedDataParallel(m)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        ddp(torch.randn(2, 8)).sum().backward()
    assert "DistributedDataParallel.forward" in {e.name for e in prof.events()}
    info = ddp.ddp_logging_data()
    assert info["exposed_comm_ms"] == -1.0  # timing off / CPU
    assert info["iterations"] == 1
