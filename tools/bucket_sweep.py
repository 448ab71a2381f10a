#!/usr/bin/env python3
"""BASELINE config #4: ResNet-50 DDP bucket-size sweep (25 MiB default vs
xGMI-tuned) at N GPUs. Launches bench.py once per (first, cap) point through
torch.distributed.run and prints one JSON line per point.

    python tools/bucket_sweep.py --gpus 8 --caps 4 8 16 25 50 100 --firsts 0.25 1 4
"""
import argparse
import itertools
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--caps", type=float, nargs="+", default=[4, 8, 16, 25, 50, 100])
    ap.add_argument("--firsts", type=float, nargs="+", default=[1.0])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--comm-dtype", default="fp32")
    ap.add_argument("--impl", default="ours")
    a = ap.parse_args()
    for first, cap in itertools.product(a.firsts, a.caps):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(a.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(29700 + int(cap * 10) % 200),
               os.path.join(REPO, "bench.py"), "--gpus", str(a.gpus), "--steps", str(a.steps), "--warmup",
               str(a.warmup), "--bucket-cap-mb", str(cap), "--first-bucket-mb", str(first), "--comm-dtype",
               a.comm_dtype, "--impl", a.impl]
        r = subprocess.run(cmd, capture_output=True, text=True)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        rec = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
        rec["sweep"] = {"first_mb": first, "cap_mb": cap}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
