"""The GPT-2 LM-head forward + loss candidates of ops/lm_head.py timed alone:
pp_xent (GEMM with the softmax partials in its epilogue + merge), pp + the
one-pass cross-entropy, hipBLASLt + the same pass. Candidates alternate call
by call (median of --calls per candidate), back to back and with a 1 ms spin
before each call. Run under two builds (PYTHONPATH) for an A/B.

    python tools/head_xent_probe.py [--calls 24] [--tag new]
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.environ.get("PROBE_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402


def run(cands, calls, spin=0):
    names = list(cands)
    ev = {k: [] for k in names}
    for i in range(calls):
        for j in range(len(names)):
            k = names[(i + j) % len(names)]
            if spin:
                torch.cuda._sleep(spin)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            cands[k]()
            e.record()
            ev[k].append((s, e))
    e.synchronize()
    return {k: statistics.median(s.elapsed_time(e) * 1e3 for s, e in v) for k, v in ev.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=24)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, V, Vp, K = 8192, 50257, 50304, 768
    g = torch.Generator(device=dev).manual_seed(0)
    x2 = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    wb = (torch.randn(Vp, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    wb[V:] = 0
    tg = torch.randint(0, V, (M,), device=dev, generator=g)
    cands = {
        "pp_xent": lambda: _C.lm_head_xent_fwd(x2, wb, tg, -100, V),
        "pp": lambda: _C.cross_entropy_fwd(_C.gemm_pp(x2, wb, None, 0)[0], tg, -100, 0.0, V),
        "hipblaslt": lambda: _C.cross_entropy_fwd(F.linear(x2, wb), tg, -100, 0.0, V),
    }
    # the candidates agree on the loss
    ref = cands["hipblaslt"]()[0].float()
    got = cands["pp_xent"]()[1].float() if len(cands["pp_xent"]()) > 2 else None
    for f in cands.values():
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(10_000_000)
    e.record()
    e.synchronize()
    spin = int(10_000_000 / max(s.elapsed_time(e), 1e-3))
    for sched in ("b2b", "gap", "b2b"):
        ts = run(cands, a.calls, spin if sched == "gap" else 0)
        print(json.dumps({"tag": a.tag, "schedule": sched, **{k: round(v, 1) for k, v in ts.items()},
                          "loss_maxdiff": None if got is None else float((got - ref).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
