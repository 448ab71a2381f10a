"""Per-kernel statistics from a rocprofv3 rocpd SQLite database (the default
output format on this image when no --output-format is given).

    python tools/rocpd_stats.py gpurun_out/x/run_results.db [NAME_REGEX] [--by-grid]

Prints calls, mean / total µs per kernel (short template-stripped name unless
the regex asks for more); --by-grid splits each kernel by its launch grid
(e.g. the BERT and GPT-2 attention shapes of tools/attn_bench.py).
"""
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main():
    db = sys.argv[1]
    args = [a for a in sys.argv[2:] if not a.startswith("--")]
    pat = re.compile(args[0]) if args else None
    by_grid = "--by-grid" in sys.argv
    c = sqlite3.connect(db)
    agg = defaultdict(list)
    for name, dur, gx, gy, gz in c.execute("select name, duration, grid_x, grid_y, grid_z from kernels"):
        if pat and not pat.search(name):
            continue
        key = (short(name), (gx, gy, gz) if by_grid else None)
        agg[key].append(dur / 1e3)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'calls':>6} {'mean us':>9} {'total us':>10}  kernel")
    for (n, g), d in rows:
        print(f"{len(d):6d} {sum(d) / len(d):9.1f} {sum(d):10.1f}  {n}" + (f"  grid={g}" if g else ""))


if __name__ == "__main__":
    main()
