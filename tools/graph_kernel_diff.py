"""Per-step kernel multiset of two rocprofv3 runs of the same workload —
eager vs whole-step HIP-graph replay (bench.py --graph 0/1) — and their
difference: which launches the captured step adds or drops, and the GPU time
of each kernel family per step in both.

The step window: the optimizer's launches close every step in both modes;
they are clustered (gap > 1 ms starts a new cluster) and the last N+1
clusters bound N steps.

    python tools/graph_kernel_diff.py eager.db graph.db [--steps 4] [--opt adam]
"""
import argparse
import sqlite3
from collections import Counter, defaultdict

from kernel_stats import short


def per_step(path, steps, opt):
    con = sqlite3.connect(path)
    ks = sorted((s, e, short(n)) for n, s, e in con.execute("select name, start, end from kernels"))
    opt_t = [(s, e) for s, e, n in ks if opt in n.lower()]
    clusters = []
    for s, e in opt_t:
        if clusters and s - clusters[-1][1] < 1_000_000:
            clusters[-1][1] = e
        else:
            clusters.append([s, e])
    if len(clusters) < steps + 1:
        raise SystemExit(f"{path}: only {len(clusters)} optimizer clusters")
    t0, t1 = clusters[-(steps + 1)][1], clusters[-1][1]
    cnt, tim = Counter(), defaultdict(float)
    busy = 0
    for s, e, n in ks:
        if s > t0 and e <= t1:
            cnt[n] += 1
            tim[n] += (e - s) / 1e3
            busy += e - s
    return ({k: v / steps for k, v in cnt.items()}, {k: v / steps for k, v in tim.items()}, (t1 - t0) / 1e6 / steps,
            busy / (t1 - t0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("eager")
    ap.add_argument("graph")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--opt", default="adam")
    a = ap.parse_args()
    ce, te, se, be = per_step(a.eager, a.steps, a.opt)
    cg, tg, sg, bg = per_step(a.graph, a.steps, a.opt)
    print(f"# per step: eager {se:.3f} ms ({sum(ce.values()):.0f} launches, kernels {sum(te.values()) / 1e3:.3f} ms, "
          f"busy {be:.3f}) | graph {sg:.3f} ms ({sum(cg.values()):.0f} launches, kernels {sum(tg.values()) / 1e3:.3f} ms, "
          f"busy {bg:.3f})")
    print(f"# {'kernel':70s} {'n_eager':>8s} {'n_graph':>8s} {'us_eager':>9s} {'us_graph':>9s}")
    names = sorted(set(ce) | set(cg), key=lambda k: -abs(tg.get(k, 0) - te.get(k, 0)))
    for k in names:
        if abs(ce.get(k, 0) - cg.get(k, 0)) < 1e-9 and abs(te.get(k, 0) - tg.get(k, 0)) < 5:
            continue
        print(f"  {k[:70]:70s} {ce.get(k, 0):8.2f} {cg.get(k, 0):8.2f} {te.get(k, 0):9.1f} {tg.get(k, 0):9.1f}")


if __name__ == "__main__":
    main()
