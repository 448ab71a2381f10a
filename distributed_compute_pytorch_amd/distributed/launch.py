"""Process launchers.

* :func:`spawn` — ``mp.spawn`` replacement (reference: main.py:150,
  SURVEY §2b F1): start ``nprocs`` interpreters with the spawn start method,
  call ``fn(i, *args)`` in each, and when one child fails terminate the rest
  and re-raise its error in the parent.
* :func:`launch_env` — torchrun-style: run a command ``nproc`` times with
  RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set; a failing
  rank tears the whole job down (SURVEY §5.3 clean abort propagation).
  CLI: ``python -m distributed_compute_pytorch_amd.distributed.run``.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import time
import traceback
from typing import Callable, List, Optional, Sequence


class ProcessRaisedException(RuntimeError):
    def __init__(self, msg: str, error_index: int, pid: int):
        super().__init__(msg)
        self.error_index = error_index
        self.pid = pid


class ProcessExitedException(RuntimeError):
    def __init__(self, msg: str, error_index: int, pid: int, exit_code: int):
        super().__init__(msg)
        self.error_index = error_index
        self.pid = pid
        self.exit_code = exit_code


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wrap(fn, i, args, err_q):
    try:
        fn(i, *args)
    except KeyboardInterrupt:
        pass
    except Exception:
        err_q.put((i, traceback.format_exc()))
        sys.exit(1)


def spawn(fn: Callable, args: Sequence = (), nprocs: int = 1, join: bool = True, daemon: bool = False,
          start_method: str = "spawn", timeout: Optional[float] = None):
    """Start ``nprocs`` processes running ``fn(rank, *args)``.

    Returns the list of processes when ``join=False``. With ``join=True`` waits
    for all; the first failure terminates the others and raises
    :class:`ProcessRaisedException` (child raised) or
    :class:`ProcessExitedException` (child died, e.g. by a signal).
    """
    ctx = mp.get_context(start_method)
    err_q = ctx.SimpleQueue()
    procs = []
    for i in range(nprocs):
        p = ctx.Process(target=_wrap, args=(fn, i, tuple(args), err_q), daemon=daemon)
        p.start()
        procs.append(p)
    if not join:
        return procs
    deadline = None if timeout is None else time.monotonic() + timeout
    alive = set(range(nprocs))
    try:
        while alive:
            for i in list(alive):
                p = procs[i]
                p.join(timeout=0.05)
                if p.exitcode is None:
                    continue
                alive.discard(i)
                if p.exitcode != 0:
                    for q in procs:
                        if q.is_alive():
                            q.terminate()
                    for q in procs:
                        q.join(timeout=10)
                        if q.is_alive():
                            q.kill()
                    if not err_q.empty():
                        idx, tb = err_q.get()
                        raise ProcessRaisedException(
                            f"\n\n-- Process {idx} terminated with the following error:\n{tb}", idx, procs[idx].pid)
                    sig = -p.exitcode if p.exitcode < 0 else None
                    what = f"signal {signal.Signals(sig).name}" if sig else f"exit code {p.exitcode}"
                    raise ProcessExitedException(f"process {i} terminated with {what}", i, p.pid, p.exitcode)
            if deadline is not None and time.monotonic() > deadline:
                for q in procs:
                    if q.is_alive():
                        q.kill()
                raise TimeoutError(f"spawn: processes did not finish within {timeout}s")
    finally:
        for q in procs:
            if q.is_alive():
                q.kill()
    return None


def launch_env(cmd: List[str], nproc: int, master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
               extra_env: Optional[dict] = None, timeout: Optional[float] = None) -> int:
    """Run ``cmd`` as ``nproc`` ranks; returns the job's exit code."""
    port = master_port or free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc),
                    "LOCAL_WORLD_SIZE": str(nproc), "MASTER_ADDR": master_addr, "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    deadline = None if timeout is None else time.monotonic() + timeout
    code = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                code = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if deadline is not None and time.monotonic() > deadline:
                code = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    return code
