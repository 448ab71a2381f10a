"""The long kernels of a rocprofv3 kernel trace in launch order, with the
gap before each one and the kernels that overlapped it on other queues — to
see what a first-call autotune window (tools/head_wgrad_probe.py's question:
why the LM-head weight gradient times 770 µs inside the GPT-2 step's
autotune and ~670 µs in isolation) contains besides the timed kernels.

    python tools/long_kernel_trace.py RUN_results.db [--min-us 300] [--window N] [--match REGEX]

--window N: also dump the N kernels (all lengths) that follow the first
kernel matching --match, with start offsets, so the autotune's interleaved
candidate calls and anything between them are visible.
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].split("<")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-us", type=float, default=300.0)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--match", default="wgrad")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    sel = f"select name, start, end, {q or '0'}, grid_x, grid_y, grid_z from kernels order by start"
    ks = [(short(n), s, e, qq, (gx, gy, gz)) for n, s, e, qq, gx, gy, gz in c.execute(sel)]
    print(f"{len(ks)} kernels; queue column: {q}")
    t0 = ks[0][1]
    prev_end = t0
    longs = []
    for i, (n, s, e, qq, g) in enumerate(ks):
        if (e - s) / 1e3 >= a.min_us:
            longs.append(i)
    print(f"{'idx':>6} {'t ms':>9} {'dur us':>8} {'gap us':>7} {'ovl us':>7} q  kernel / grid / overlapping")
    for i in longs:
        n, s, e, qq, g = ks[i]
        gap = (s - ks[i - 1][2]) / 1e3 if i else 0.0
        ov, names = 0.0, set()
        j = i - 1
        while j >= 0 and ks[j][2] > s - 10_000_000:  # earlier kernels still running
            if ks[j][3] != qq and ks[j][2] > s:
                ov += (min(e, ks[j][2]) - s) / 1e3
                names.add(ks[j][0])
            j -= 1
        j = i + 1
        while j < len(ks) and ks[j][1] < e:
            if ks[j][3] != qq:
                ov += (min(e, ks[j][2]) - ks[j][1]) / 1e3
                names.add(ks[j][0])
            j += 1
        print(f"{i:6d} {(s - t0) / 1e6:9.3f} {(e - s) / 1e3:8.1f} {gap:7.1f} {ov:7.1f} {qq} {n} {g} "
              f"{sorted(names)[:4] if names else ''}")
    if a.window:
        pat = re.compile(a.match)
        first = next((i for i in longs if pat.search(ks[i][0])), None)
        if first is None:
            print("no long kernel matches", a.match)
            return
        print(f"\nwindow: {a.window} kernels from #{first}")
        base = ks[first][1]
        for n, s, e, qq, g in ks[first:first + a.window]:
            print(f"{(s - base) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {qq} {n} {g}")


if __name__ == "__main__":
    main()
