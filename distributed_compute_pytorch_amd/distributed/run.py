"""torchrun-style launcher CLI.

    python -m distributed_compute_pytorch_amd.distributed.run --nproc-per-node 8 train.py --args

Each rank gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT; the
first failing rank terminates the job (exit code propagated).
"""
from __future__ import annotations

import argparse
import sys

from .launch import launch_env


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    ap.add_argument("--master-port", "--master_port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("-m", dest="module", action="store_true", help="run the target as a module")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable] + (["-m", a.script] if a.module else [a.script]) + a.script_args
    sys.exit(launch_env(cmd, a.nproc_per_node, a.master_addr, a.master_port, timeout=a.timeout))


if __name__ == "__main__":
    main()
