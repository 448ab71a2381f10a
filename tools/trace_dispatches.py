"""Per-dispatch kernel durations from a rocprofv3 --kernel-trace CSV directory,
in launch order (name truncated, grid size, us): what a per-shape probe ran.

    python tools/trace_dispatches.py <rocprofv3 -d dir> [NAME_REGEX]
"""
import csv
import glob
import os
import re
import sys


def main():
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    rows = []
    for p in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if pat.search(r["Kernel_Name"]):
                rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "?")),
                             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    for _, k, g, us in sorted(rows):
        print(f"{us:9.1f}  grid={g:>8}  {k[:120]}")


if __name__ == "__main__":
    main()
