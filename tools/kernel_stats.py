"""Per-kernel call count / mean / total time from a rocprofv3 run (rocpd
SQLite database or kernel-trace CSV), optionally with the grid size so that
one kernel's different shapes separate.

    python tools/kernel_stats.py <prof_results.db | kernel_trace.csv> [--top 30] [--grid]
    python tools/kernel_stats.py <db> --families --steps N   # GPU us per step per kernel family
"""
import argparse
import csv
import sqlite3
from collections import defaultdict


def short(name):
    """kernel name without its parameter list (template arguments kept)"""
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0:
            return name[:i]
    return name


def rows(path, grid):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
        gcols = [c for c in cols if "grid" in c.lower()][:3] if grid else []
        gsel = "".join(", " + c for c in gcols)
        for rec in con.execute(f"select name, start, end{gsel} from kernels"):
            yield (("grid=" + "x".join(str(v) for v in rec[3:]) + " " if gcols else "") + short(rec[0]),
                   rec[2] - rec[1])
    else:
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if grid:
                n = f"grid={r.get('Grid_Size_X')}x{r.get('Grid_Size_Y')}x{r.get('Grid_Size_Z')} " + short(n)
            yield n, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--families", action="store_true", help="group by kernel name without template arguments")
    ap.add_argument("--steps", type=int, default=1, help="divide family totals by this many steps")
    ap.add_argument("--busy", type=float, default=None, metavar="SKIP",
                    help="GPU busy fraction (union of kernel intervals / span) after skipping the first SKIP of the span")
    ap.add_argument("--window", default=None, metavar="NAME:N",
                    help="with --busy: the window between the last N launches of kernel NAME (substring)")
    a = ap.parse_args()
    if a.busy is not None:
        con = sqlite3.connect(a.path)
        iv = sorted(con.execute("select start, end from kernels"))
        t0, t1 = iv[0][0], max(e for _, e in iv)
        cut = t0 + a.busy * (t1 - t0)
        if a.window:
            name, n = a.window.rsplit(":", 1)
            starts = sorted(st for nm, st in con.execute("select name, start from kernels") if name in nm)[-int(n):]
            cut, t1 = starts[0], starts[-1]
            iv = [(max(s_, cut), min(e_, t1)) for s_, e_ in iv if e_ > cut and s_ < t1]
        busy, cur_s, cur_e = 0, None, None
        for s_, e_ in iv:
            if e_ <= cut:
                continue
            s_ = max(s_, cut)
            if cur_e is None or s_ > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s_, e_
            else:
                cur_e = max(cur_e, e_)
        busy += cur_e - cur_s
        print(f"# GPU busy {busy / (t1 - cut):.3f} of {(t1 - cut) / 1e6:.1f} ms "
              f"({'window ' + a.window if a.window else f'first {a.busy:.0%} of the trace skipped'})")
        return
    if a.families:
        fam = defaultdict(float)
        for n, d in rows(a.path, False):
            base = n.split("<")[0].split("::")[-1].strip()
            fam[base] += d
        tot = sum(fam.values())
        print(f"# GPU time per step per kernel family, us (share); {tot / a.steps / 1e3:.1f} us per step")
        for n, t in sorted(fam.items(), key=lambda kv: -kv[1])[: a.top]:
            print(f"  {t / a.steps / 1e3:9.1f}  {100 * t / tot:4.1f}%  {n[:60]}")
        return
    agg = defaultdict(lambda: [0, 0])
    for n, d in rows(a.path, a.grid):
        agg[n][0] += 1
        agg[n][1] += d
    print(f"{'calls':>6} {'mean us':>9} {'total ms':>9}  kernel")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{c:6d} {t / c / 1e3:9.1f} {t / 1e6:9.2f}  {n[:150]}")


if __name__ == "__main__":
    main()
