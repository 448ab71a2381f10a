"""Summarise a rocprofv3 `--pmc <COUNTER> --kernel-trace --output-format csv`
run: per kernel name, mean duration and mean counter value, and the implied
bandwidth (counter bytes / duration) for FETCH_SIZE / WRITE_SIZE (KiB units).

    python tools/pmc_summary.py <dir with *_counter_collection.csv and *_kernel_trace.csv> [--top 30]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    cc = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        raise SystemExit("no counter_collection.csv under " + a.dir)
    dur = {}
    for path in kt:
        for r in csv.DictReader(open(path)):
            dur[_col(r, "Dispatch_Id", "Dispatch_ID")] = (int(_col(r, "End_Timestamp")) -
                                                          int(_col(r, "Start_Timestamp"))) / 1e3  # us
    agg = defaultdict(lambda: defaultdict(lambda: [0, 0.0, 0.0]))
    for path in cc:
        for r in csv.DictReader(open(path)):
            name = _col(r, "Kernel_Name")
            cn = _col(r, "Counter_Name")
            v = float(_col(r, "Counter_Value"))
            d = dur.get(_col(r, "Dispatch_Id", "Dispatch_ID"), 0.0)
            e = agg[name][cn]
            e[0] += 1
            e[1] += v
            e[2] += d
    rows = []
    for name, cs in agg.items():
        for cn, (n, v, d) in cs.items():
            rows.append((d / n, name, cn, v / n))
    rows.sort(key=lambda t: -t[0] * 1)
    print(f"{'us/call':>9} {'counter':>11} {'value/call':>12} {'GB/s':>8}  kernel")
    for us, name, cn, v in rows[: a.top]:
        bw = v * 1024 / (us * 1e-6) / 1e9 if cn in ("FETCH_SIZE", "WRITE_SIZE") and us > 0 else float("nan")
        print(f"{us:9.1f} {cn:>11} {v:12.1f} {bw:8.0f}  {name[:100]}")


if __name__ == "__main__":
    main()
