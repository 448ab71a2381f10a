"""Long host-side HIP API calls in a rocprofv3 --hip-trace CSV run (the calls
that block the host and let the GPU queue drain): in the window between the
first and last of the last N launches of kernel NAME, per API function the
calls longer than --min-us, their count and total time, plus the kernels that
ran just before / after the longest ones.

    python tools/hip_api_stalls.py <dir with *_hip_api_trace.csv and *_kernel_trace.csv> --window xent_fwd:20
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window", required=True)
    ap.add_argument("--min-us", type=float, default=50.0)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    kf = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    hf = glob.glob(os.path.join(a.dir, "**", "*hip_api_trace.csv"), recursive=True)
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for f in kf
                for r in csv.DictReader(open(f)))
    name, n = a.window.rsplit(":", 1)
    starts = [s for s, _, k in ks if name in k][-int(n):]
    t0, t1 = starts[0], starts[-1]
    calls = []
    for f in hf:
        for r in csv.DictReader(open(f)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s >= t0 and e <= t1:
                calls.append((s, e, r.get("Function") or r.get("Operation") or "?"))
    agg = defaultdict(lambda: [0, 0.0])
    long = []
    for s, e, fn in calls:
        d = (e - s) / 1e3
        if d >= a.min_us:
            agg[fn][0] += 1
            agg[fn][1] += d
            long.append((d, s, fn))
    print(f"# window {(t1 - t0) / 1e6:.1f} ms, {len(calls)} HIP API calls; calls >= {a.min_us} us:")
    for fn, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{t / a.steps:10.0f} us/step {c / a.steps:7.1f} calls/step  {fn}")
    cf = glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    copies = []
    for f in cf:
        for r in csv.DictReader(open(f)):
            s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s_ >= t0 and e_ <= t1:
                copies.append((s_, e_, r.get("Direction") or r.get("Operation") or "copy"))
    gaps_detail(ks, calls, copies, t0, t1)
    long.sort(reverse=True)
    kstarts = [s for s, _, _ in ks]
    import bisect
    print("# longest calls: previous / next kernel start")
    for d, s, fn in long[:15]:
        i = bisect.bisect_left(kstarts, s)
        prev = ks[i - 1][2][:60] if i > 0 else "-"
        nxt = ks[i][2][:60] if i < len(ks) else "-"
        print(f"{d:9.0f} us  {fn:32s} after {prev}  before {nxt}")


def gaps_detail(ks, calls, copies, t0, t1, top=4):
    """The largest kernel-free intervals and the HIP calls / copies around them."""
    gaps, cur_end, prev = [], None, None
    for s, e, k in ks:
        if e <= t0 or s >= t1:
            continue
        if cur_end is not None and s > cur_end:
            gaps.append((s - cur_end, cur_end, s, prev, k))
        if cur_end is None or e > cur_end:
            cur_end, prev = e, k
    gaps.sort(reverse=True)
    for g, gs, ge, pk, nk in gaps[:top]:
        print(f"# gap {g / 1e3:.0f} us: after {pk[:50]} before {nk[:50]}")
        for s, e, fn in sorted(c for c in calls if gs - 300000 <= c[0] <= ge):
            if (e - s) >= 5000 or gs <= s:
                print(f"    api {(s - gs) / 1e3:+9.1f} us  {(e - s) / 1e3:8.1f} us  {fn}")
        for s, e, fn in sorted(c for c in copies if gs - 300000 <= c[0] <= ge):
            print(f"    copy {(s - gs) / 1e3:+8.1f} us  {(e - s) / 1e3:8.1f} us  {fn}")


if __name__ == "__main__":
    main()
