"""Worker for tests/test_gpu_rccl_fault.py (a fresh child process: the
communicator reads DCP_SINGLE_RANK_HOP at construction).

Drives the RCCL failure path on ONE GPU: a 1-rank RCCL
communicator in single-rank-hop mode (collectives on the comm stream with
per-Work deadlines) with a 1.5 s timeout. A bounded spin kernel (~4 s) on the
caller's stream stalls a comm-stream fence exactly like a hung collective;
the watchdog must hit the deadline, ncclCommAbort the communicator, and
Work.synchronize() must raise "timed out" within ~timeout + one poll, long
before the spin ends. Afterwards every Work / collective raises. Nothing of
RCCL is queued behind the stall (the fence issues no collective), so the
abort never races a launched RCCL kernel. Prints one FAULTRESULT JSON line.
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from distributed_compute_pytorch_amd._ext import C

    assert os.environ.get("DCP_SINGLE_RANK_HOP") == "1"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    res = {}
    store = C.TCPStore("127.0.0.1", 0, 1, True, 30000, False)
    timeout_ms = 1500
    comm = C.make_rccl_communicator(store, "fault", 0, 1, 0, timeout_ms)
    x = torch.ones(4096, device=dev)
    comm.all_reduce(x, C.ReduceOp.SUM).synchronize()  # healthy first
    res["healthy_ok"] = bool((x == 1).all().item()) and comm.error() == ""

    # calibrate the spin: cycles per ms of torch.cuda._sleep on this device
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    torch.cuda._sleep(20_000_000)
    e.record()
    torch.cuda.synchronize()
    per_ms = 20_000_000 / max(s.elapsed_time(e), 1e-3)
    spin_ms = 4000.0
    res["spin_cycles_per_ms"] = per_ms

    torch.cuda._sleep(int(per_ms * spin_ms))  # caller stream stalled ~4 s
    w = comm.stream_fence()
    t0 = time.time()
    try:
        w.synchronize()
        res["raised"] = False
    except Exception as ex:  # TimeoutError / RuntimeError from the watchdog abort
        res["raised"] = True
        res["message"] = str(ex)[:300]
    res["raise_after_s"] = round(time.time() - t0, 3)
    res["error"] = comm.error()[:300]
    after = {}
    for name, fn in (("is_completed", w.is_completed), ("wait", w.wait),
                     ("all_reduce", lambda: comm.all_reduce(x, C.ReduceOp.SUM))):
        try:
            fn()
            after[name] = False
        except Exception:
            after[name] = True
    res["raises_after_abort"] = after
    res["timeout_ms"] = timeout_ms
    res["spin_ms"] = spin_ms
    print("FAULTRESULT " + json.dumps(res), flush=True)
    # the spin kernel still drains (bounded) before the process exits


if __name__ == "__main__":
    main()
