"""Launcher semantics: error propagation and fault injection."""
import os
import subprocess
import sys
import textwrap
import time

import pytest

from distributed_compute_pytorch_amd.distributed.launch import (ProcessExitedException, ProcessRaisedException,
                                                                 launch_env, spawn)


def _ok(rank, out_dir):
    open(os.path.join(out_dir, f"r{rank}"), "w").write(str(rank))


def _boom(rank):
    if rank == 1:
        raise ValueError("injected failure on rank 1")
    time.sleep(60)


def _die(rank):
    if rank == 0:
        os._exit(7)
    time.sleep(60)


def test_spawn_runs_all(tmp_path):
    spawn(_ok, (str(tmp_path),), nprocs=3)
    assert sorted(os.listdir(tmp_path)) == ["r0", "r1", "r2"]


def test_spawn_propagates_exception_and_kills_peers():
    t0 = time.time()
    with pytest.raises(ProcessRaisedException, match="injected failure"):
        spawn(_boom, (), nprocs=3)
    assert time.time() - t0 < 40


def test_spawn_reports_exit_code():
    with pytest.raises(ProcessExitedException) as e:
        spawn(_die, (), nprocs=2)
    assert e.value.exit_code == 7


def test_launch_env_fault_injection(tmp_path):
    """Kill one rank mid-collective: the whole job must exit with an error quickly
    instead of hanging in the collective."""
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, time, datetime
        sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})
        import torch
        import distributed_compute_pytorch_amd.distributed as dist
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=20))
        r = dist.get_rank()
        t = torch.ones(4)
        dist.all_reduce(t)
        if r == 1:
            os._exit(3)   # injected crash
        for _ in range(100):
            dist.all_reduce(t)
            time.sleep(0.1)
    """))
    t0 = time.time()
    code = launch_env([sys.executable, str(script)], 3, timeout=120)
    assert code != 0
    assert time.time() - t0 < 60


def test_torchrun_agent_store_compat(tmp_path):
    """Under torch.distributed.run the elastic agent already listens on
    MASTER_PORT (TORCHELASTIC_USE_AGENT_STORE=True): our store must bootstrap
    through it instead of binding the same port (this is how the driver
    launches the multi-GPU bench)."""
    from distributed_compute_pytorch_amd.distributed.launch import free_port

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {repo!r})
        import torch, torch.nn.functional as F
        import distributed_compute_pytorch_amd as dcp
        from distributed_compute_pytorch_amd.models import ConvNet
        dcp.distributed.init_process_group("gloo")
        r, w = dcp.distributed.get_rank(), dcp.distributed.get_world_size()
        torch.manual_seed(0)
        m = dcp.parallel.DistributedDataParallel(ConvNet())
        F.nll_loss(m(torch.randn(4, 1, 28, 28) + r), torch.zeros(4, dtype=torch.long)).backward()
        g = m.module.fc1.weight.grad.clone()
        ref = g.clone(); dcp.distributed.broadcast(ref, 0)
        assert torch.allclose(g, ref), "replicas diverged"
        t = torch.tensor([float(r)]); dcp.distributed.all_reduce(t)
        assert t.item() == sum(range(w))
        dcp.distributed.destroy_process_group()
        print("OK", r)
    """))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "3",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(script)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("OK") == 3
