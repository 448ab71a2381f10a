"""RCCL failure detection on one GPU: watchdog deadline →
ncclCommAbort → raise, in a child process (tests/gpu_fault_worker.py).
Code under test: rccl_comm.cpp watchdog(), RcclWork::synchronize / wait /
is_completed, launch()'s raise_if_error."""
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_watchdog_aborts_stalled_collective(cuda):
    env = dict(os.environ, DCP_SINGLE_RANK_HOP="1")
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_fault_worker.py")], env=env, capture_output=True,
                       text=True, timeout=120)
    wall = time.time() - t0
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("FAULTRESULT ")][-1]
    res = json.loads(line[len("FAULTRESULT "):])
    print(res, f"child wall {wall:.1f}s")
    assert res["healthy_ok"]
    assert res["raised"], res
    assert "timed out" in res["message"] and "timed out" in res["error"], res
    # raised at the deadline (+ watchdog poll), not when the ~4 s stall ended
    assert res["timeout_ms"] / 1e3 * 0.9 <= res["raise_after_s"] <= res["timeout_ms"] / 1e3 + 1.5, res
    assert res["raise_after_s"] < res["spin_ms"] / 1e3 * 0.8, res
    assert all(res["raises_after_abort"].values()), res
