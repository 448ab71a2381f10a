"""Does the LM-head weight gradient's autotune time depend on what ran just
before it (the chip's power / clock state) rather than on the kernel?

Times ours (split-M wgrad, conv1x1_wgrad) and hipBLASLt (addmm, fp32 out)
on the GPT-2 head shape, per call with event pairs, in three schedules:

* ``b2b``: the two alternate call by call, back to back (what the
  interleaved autotune does);
* ``gap``: the same, with a ~1 ms spin kernel (torch.cuda._sleep: one wave,
  little power) before every timed call — closer to the step, where the
  head GEMMs follow lighter kernels;
* ``hot``: ``b2b`` right after 300 ms of back-to-back bf16 GEMMs (the
  autotune runs in the first step, after other shapes' bursts).

    python tools/autotune_clock_probe.py [--calls 24]

One JSON line per (schedule, candidate): median / min / first-8 / last-8 µs.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def run(cands, calls, spin_cycles=0):
    names = list(cands)
    ev = {k: [] for k in names}
    for i in range(calls):
        for j in range(len(names)):
            k = names[(i + j) % len(names)]
            if spin_cycles:
                torch.cuda._sleep(spin_cycles)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            cands[k]()
            e.record()
            ev[k].append((s, e))
    e.synchronize()
    return {k: [s.elapsed_time(e) * 1e3 for s, e in v] for k, v in ev.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=24)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, V, Vp, K = 8192, 50257, 50304, 768
    g = torch.Generator(device=dev).manual_seed(0)
    x2 = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    logits = (torch.randn(M, Vp, device=dev, generator=g) * 2).to(torch.bfloat16)
    tg = torch.randint(0, V, (M,), device=dev, generator=g)
    _, lse = _C.cross_entropy_fwd(logits, tg, -100, 0.0, V)
    d = _C.cross_entropy_bwd(logits, tg, lse, torch.full((1,), 1.0 / M, device=dev), -100, 0.0, V, True)
    acc = torch.zeros(V, K, device=dev)
    cands = {
        "ring": lambda: _C.conv1x1_wgrad(d, x2, accumulate_into=acc, out_rows=V),
        "hipblaslt": lambda: torch.addmm(acc, d[:, :V].t(), x2, out_dtype=torch.float32, out=acc),
    }
    for f in cands.values():
        f()
    # ~1 ms of spin: the clock rate is read back from a timed spin
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(10_000_000)
    e.record()
    torch.cuda.synchronize()
    spin = int(10_000_000 / max(s.elapsed_time(e), 1e-3))  # cycles per ms
    ha = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for sched in ("b2b", "gap", "hot", "b2b"):
        if sched == "hot":
            t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t[0].record()
            for _ in range(300):
                ha @ ha
                t[1].record()
                if _ % 50 == 49:
                    t[1].synchronize()
                    if t[0].elapsed_time(t[1]) > 300:
                        break
        ts = run(cands, a.calls, spin if sched == "gap" else 0)
        for k, v in ts.items():
            print(json.dumps({"schedule": sched, "cand": k, "median_us": round(statistics.median(v), 1),
                              "min_us": round(min(v), 1), "first8": [round(x) for x in v[:8]],
                              "last8": [round(x) for x in v[-8:]]}), flush=True)


if __name__ == "__main__":
    main()
