"""Per (kernel, grid) group of a rocprofv3 --pmc --kernel-trace CSV run: calls,
mean µs, mean counter value, and for FETCH_SIZE / WRITE_SIZE (KiB) the
achieved TB/s — ResNet's GEMM families run one instantiation over several
shapes, which the grid size tells apart.

    python tools/pmc_by_dispatch.py <dir> [--top 30] [--match gemm_nt]
(gfx950: FETCH_SIZE counts half the bytes of wide coalesced reads —
MI355X_MICROARCH.md; the "x2" column is that correction.)
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+", help="one rocprofv3 output dir per counter pass (merged by kernel + grid)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--match", default=".")
    a = ap.parse_args()
    pat = re.compile(a.match)
    groups = defaultdict(lambda: {"n": 0, "us": 0.0, "c": defaultdict(float), "cn": defaultdict(int)})
    for pi, d in enumerate(a.dirs):
        info = {}
        for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                did = r.get("Dispatch_Id") or r.get("Dispatch_ID")
                grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
                info[did] = (r["Kernel_Name"], grid, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        vals = defaultdict(lambda: defaultdict(list))
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                did = r.get("Dispatch_Id") or r.get("Dispatch_ID")
                if did in info:
                    vals[did][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for did, (name, grid, us) in info.items():
            if not pat.search(name) or did not in vals:
                continue
            g = groups[(name, grid)]
            if pi == 0:  # durations from the first pass
                g["n"] += 1
                g["us"] += us
            for c, v in vals[did].items():
                g["c"][c] += sum(v)
                g["cn"][c] += 1
    rows = sorted(groups.items(), key=lambda kv: -kv[1]["us"])[:a.top]
    # FETCH + WRITE together where both passes ran: the kernel's HBM-side traffic rate
    for (name, grid), g in rows:
        n, us = g["n"], g["us"] / g["n"]
        parts = [f"{n:4d} x {us:8.1f} us grid={grid:>8}"]
        if n == 0:
            continue
        for c, tot in sorted(g["c"].items()):
            v = tot / g["cn"][c]
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                tbs = v * 1024 / (us * 1e-6) / 1e12
                parts.append(f"{c}={v / 1024:.1f}MiB {tbs:.2f}TB/s" + (f" (x2 {2 * tbs:.2f})" if c == "FETCH_SIZE" else ""))
            else:
                parts.append(f"{c}={v:.3g}")
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[-90:]
        if "FETCH_SIZE" in g["c"] and "WRITE_SIZE" in g["c"]:
            tot = (2 * g["c"]["FETCH_SIZE"] / g["cn"]["FETCH_SIZE"] + g["c"]["WRITE_SIZE"] / g["cn"]["WRITE_SIZE"]) * 1024
            parts.append(f"total(x2 fetch)={tot / (us * 1e-6) / 1e12:.2f}TB/s")
        print("  ".join(parts) + "  " + short)


if __name__ == "__main__":
    main()
