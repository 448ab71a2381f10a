"""Where the GPU idles between kernels: from a rocprofv3 database, in the
window between the first and last of the last N launches of kernel NAME,
every idle interval (no kernel running) attributed to the (previous kernel,
next kernel) family pair around it; the pairs with the most idle time, with
the count and the median gap. Host-bound stretches show up as long gaps
before the same kernels each step; dependent-launch boundaries as many short
ones.

    python tools/gap_stats.py run_results.db --window xent_fwd:40 [--top 25] [--steps 10]
"""
import argparse
import sqlite3
import statistics
from collections import defaultdict

from kernel_stats import short


def family(n):
    n = short(n)
    return n.split("<")[0].split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--window", required=True, metavar="NAME:N")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    con = sqlite3.connect(a.path)
    ks = sorted((s, e, n) for n, s, e in con.execute("select name, start, end from kernels"))
    name, cnt = a.window.rsplit(":", 1)
    starts = [s for s, _, n in ks if name in n][-int(cnt):]
    t0, t1 = starts[0], starts[-1]
    gaps = defaultdict(list)
    total_gap = 0
    cur_end, prev = None, None
    for s, e, n in ks:
        if e <= t0 or s >= t1:
            continue
        if cur_end is not None and s > cur_end:
            g = s - cur_end
            gaps[(family(prev), family(n))].append(g)
            total_gap += g
        if cur_end is None or e > cur_end:
            cur_end, prev = e, n
    span = t1 - t0
    print(f"# window {span / 1e6:.1f} ms, idle {total_gap / 1e6:.2f} ms ({total_gap / span:.1%}), "
          f"{sum(len(v) for v in gaps.values())} gaps; per step ({a.steps}): idle {total_gap / 1e3 / a.steps:.0f} us")
    print(f"{'idle us/step':>12} {'gaps/step':>9} {'median us':>9}  prev -> next")
    for (p, nx), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        print(f"{sum(v) / 1e3 / a.steps:12.0f} {len(v) / a.steps:9.1f} {statistics.median(v) / 1e3:9.2f}  {p} -> {nx}")


if __name__ == "__main__":
    main()
