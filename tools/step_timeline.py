"""In-order kernel timeline of ONE optimizer step from a rocprofv3 kernel trace
(rocpd SQLite .db or kernel_trace.csv): name, grid, duration, gap to the
previous kernel — to attribute kernel time to layers.

    python tools/step_timeline.py prof_results.db [--marker mt_sgd] [--step -2] [--group]

--group: totals per (short name, grid) over the chosen step instead of the list.
"""
import argparse
import csv
import sqlite3
from collections import defaultdict

from kernel_stats import short


def load(path):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
        want = ["name", "start", "end"]
        grid = [c for c in ("grid_size_x", "grid_x", "grid_size", "workgroup_size_x") if c in cols]
        q = "select " + ", ".join(want + grid[:1]) + " from kernels"
        out = []
        for r in con.execute(q):
            out.append({"name": r[0], "start": int(r[1]), "end": int(r[2]), "grid": r[3] if grid else ""})
        return out
    out = []
    for r in csv.DictReader(open(path)):
        g = r.get("Grid_Size_X") or r.get("Grid_Size") or r.get("Grid_Sizes") or ""
        out.append({"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                    "grid": g})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="mt_sgd_kernel")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over marker intervals)")
    ap.add_argument("--group", action="store_true")
    a = ap.parse_args()
    rows = sorted(load(a.path), key=lambda r: r["start"])
    marks = [i for i, r in enumerate(rows) if a.marker in r["name"]]
    spans = [(marks[k] + 1, marks[k + 1] + 1) for k in range(len(marks) - 1)]
    lo, hi = spans[a.step]
    step = rows[lo:hi]
    wall = (step[-1]["end"] - step[0]["start"]) / 1e6
    busy = sum(r["end"] - r["start"] for r in step) / 1e6
    print(f"# step {a.step}: {len(step)} kernels, wall {wall:.3f} ms, kernel sum {busy:.3f} ms")
    if a.group:
        agg = defaultdict(lambda: [0, 0.0])
        for r in step:
            k = (short(r["name"])[:110], r["grid"])
            agg[k][0] += 1
            agg[k][1] += (r["end"] - r["start"]) / 1e3
        for (n, g), (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{us:9.1f} us {c:3d}x grid={g!s:>7}  {n}")
        return
    prev = None
    for r in step:
        gap = (r["start"] - prev) / 1e3 if prev else 0.0
        prev = r["end"]
        print(f"{(r['end'] - r['start']) / 1e3:8.1f} us  gap {gap:6.1f}  grid={r['grid']!s:>7}  {short(r['name'])[:120]}")


if __name__ == "__main__":
    main()
