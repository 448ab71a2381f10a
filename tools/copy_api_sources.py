"""Which HIP API calls launch the runtime's blit kernels (``__amd_rocclr_*``)?

Reads a ``rocprofv3 --hip-trace --kernel-trace --output-format csv`` directory
(tools/hip_stalls.sh) and joins every blit-kernel dispatch to the HIP API
call with the same correlation id: counts per (kernel, API function), plus
the kernels launched right before and after (what the copy sits between).

    python tools/copy_api_sources.py /tmp/<trace dir> [--steps N]
"""
import argparse
import csv
import glob
import os
from collections import Counter


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    kf = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    hf = glob.glob(os.path.join(a.dir, "**", "*hip_api_trace.csv"), recursive=True)
    ks = sorted((int(r["Start_Timestamp"]), r["Kernel_Name"], r.get("Correlation_Id", "")) for f in kf
                for r in csv.DictReader(open(f)))
    api = {}
    for f in hf:
        for r in csv.DictReader(open(f)):
            api[r.get("Correlation_Id", "")] = r.get("Function") or r.get("Operation") or "?"
    by_api, ctx = Counter(), Counter()
    for i, (_, name, cid) in enumerate(ks):
        if not name.startswith("__amd_rocclr"):
            continue
        fn = api.get(cid, "?")
        by_api[(name, fn)] += 1
        prev = next((ks[j][1] for j in range(i - 1, -1, -1) if not ks[j][1].startswith("__amd")), "-")
        nxt = next((ks[j][1] for j in range(i + 1, len(ks)) if not ks[j][1].startswith("__amd")), "-")
        ctx[(name, fn, prev[:70], nxt[:70])] += 1
    print("# blit kernels per step by HIP API call")
    for (k, fn), c in by_api.most_common():
        print(f"{c / a.steps:8.1f}  {k:34s} {fn}")
    print("# ... and the kernels around them")
    for (k, fn, p, n), c in ctx.most_common(a.top):
        print(f"{c / a.steps:8.1f}  {k[13:]:20s} {fn:22s} after {p}  before {n}")


if __name__ == "__main__":
    main()
