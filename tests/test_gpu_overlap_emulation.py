"""Contention emulation on one GPU (parallel/comm_hooks.py
contention_emulation_hook, NOTES §22): the hook stands in for an 8-rank ring
all-reduce of each bucket on the RCCL communicator's stream. Checks, from
bench.py --comm-timing, that every bucket's collective occupied its stream for
at least the modelled time (alpha + 2(N-1)/N x bytes / busbw) and that the step
reports an exposed-communication figure. Runs bench.py in a child process:
the emulation needs DCP_SINGLE_RANK_HOP=1 before the communicator exists."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_contention_emulation_hook_runs_modelled_collectives(tmp_path, cuda):
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    busbw, world, alpha = 300.0, 8, 20.0
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--model", "resnet50", "--batch", "32",
                        "--steps", "3", "--warmup", "2", "--comm-timing", "1", "--emulate-world", str(world),
                        "--emulate-busbw", str(busbw)], capture_output=True, text=True, cwd=tmp_path, env=env,
                       timeout=400)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    assert rec["config"]["emulated_comm"]["world"] == world
    comm = rec["comm"]
    sizes = [round(b * 2**20) for b in rec["config"]["buckets_mb"]]
    assert len(comm["bucket_comm_ms"]) == len(sizes) > 1
    for nbytes, ms in zip(sizes, comm["bucket_comm_ms"]):
        model_ms = (alpha + 2 * (world - 1) / world * nbytes / (busbw * 1e3)) / 1e3
        assert ms >= 0.9 * model_ms, (nbytes, ms, model_ms)
    assert comm["exposed_comm_ms"] >= 0.0
