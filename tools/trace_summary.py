"""Summarise a rocprofv3 kernel trace over the last N optimizer steps.

A step boundary is the fused-SGD launch (or a user-given kernel-name substring).
Usage: python tools/trace_summary.py run_kernel_trace.csv|prof_results.db [--steps 5] [--marker mt_sgd]
(rocprofv3 writes a rocpd SQLite database by default; CSV with --output-format csv.)
"""
import argparse
import csv
import sqlite3
from collections import defaultdict


def _load(path):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels")]
    return list(csv.DictReader(open(path)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="mt_sgd_kernel")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = _load(a.csv)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} markers found")
    lo, hi = marks[-a.steps - 1] + 1, marks[-1] + 1
    sel = rows[lo:hi]
    t0 = int(sel[0]["Start_Timestamp"])
    t1 = int(sel[-1]["End_Timestamp"])
    wall = (t1 - t0) / 1e6 / a.steps
    agg = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = r["Kernel_Name"]
        agg[name][0] += 1
        agg[name][1] += d
        busy += d
    print(f"steps={a.steps} wall/step={wall:.3f} ms  kernel-sum/step={busy / a.steps:.3f} ms  "
          f"kernels/step={len(sel) / a.steps:.0f}")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{t / a.steps:8.3f} ms/step {n / a.steps:6.1f}/step  {100 * t / busy:5.1f}%  {name[:110]}")


if __name__ == "__main__":
    main()
