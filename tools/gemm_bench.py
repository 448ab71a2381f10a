"""1x1 convolutions at ResNet-50 b256 shapes: our MFMA GEMMs (gemm.hip) vs
MIOpen through torch (channels_last bf16), forward / dgrad / wgrad.

Reports µs per call, the analytic minimum bytes (every operand once) as
TB/s, and TFLOP/s.

    python tools/gemm_bench.py [--iters 20] [--batch 256] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_compute_pytorch_amd  # noqa: E402,F401
from distributed_compute_pytorch_amd._ext import C as _C  # noqa: E402

# (H=W, Cin, Cout): ResNet-50 stride-1 1x1 convolutions
SHAPES = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
          (14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--json", default=None)
    ap.add_argument("--no3x3", action="store_true")
    ap.add_argument("--only3x3", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    bf = torch.bfloat16
    cl = torch.channels_last
    rows = []
    for hw, ci, co in [] if a.only3x3 else SHAPES:
        M = a.batch * hw * hw
        x = torch.randn(a.batch, ci, hw, hw, device=dev).to(bf).contiguous(memory_format=cl)
        gy = torch.randn(a.batch, co, hw, hw, device=dev).to(bf).contiguous(memory_format=cl)
        w = (torch.randn(co, ci, device=dev) / ci ** 0.5).to(bf)
        w4 = w[:, :, None, None].contiguous()
        wt = w.t().contiguous()
        sc = torch.ones(ci, device=dev)
        sf = torch.zeros(ci, device=dev)
        flops = 2.0 * M * ci * co
        b_fwd = (M * (ci + co) + ci * co) * 2
        res = {"shape": f"M={M} {ci}->{co}", "M": M, "cin": ci, "cout": co}
        ours = {
            "fwd": lambda: _C.conv1x1_fwd(x, w, None, None, False, False),
            "fwd+bnrelu+stats": lambda: _C.conv1x1_fwd(x, w, sc, sf, True, True),
            "fwd+stats": lambda: _C.conv1x1_fwd(x, w, None, None, False, True),
            "fwd+bnrelu": lambda: _C.conv1x1_fwd(x, w, sc, sf, True, False),
            "dgrad": lambda: _C.conv1x1_dgrad(gy, wt),
            "wgrad": lambda: _C.conv1x1_wgrad(gy, x),
        }
        xr = x.detach().requires_grad_(False)
        miopen = {
            "fwd": lambda: F.conv2d(xr, w4),
            "dgrad": lambda: torch.ops.aten.convolution_backward(gy, xr, w4, None, (1, 1), (0, 0), (1, 1), False,
                                                                 (0, 0), 1, (True, False, False)),
            "wgrad": lambda: torch.ops.aten.convolution_backward(gy, xr, w4, None, (1, 1), (0, 0), (1, 1), False,
                                                                 (0, 0), 1, (False, True, False)),
        }
        for k, fn in ours.items():
            us = timeit(fn, a.iters)
            res[f"ours_{k}_us"] = round(us, 1)
            res[f"ours_{k}_TBps"] = round(b_fwd / (us * 1e-6) / 1e12, 2)
            res[f"ours_{k}_TFps"] = round(flops / (us * 1e-6) / 1e12, 1)
        for k, fn in miopen.items():
            us = timeit(fn, a.iters)
            res[f"miopen_{k}_us"] = round(us, 1)
            res[f"miopen_{k}_TBps"] = round(b_fwd / (us * 1e-6) / 1e12, 2)
        rows.append(res)
        print(json.dumps(res), flush=True)
    # 3x3 weight gradients (ResNet-50 conv2 layers): gathered implicit GEMM vs MIOpen
    for hw, c, st in [] if a.no3x3 else [(56, 64, 1), (56, 128, 2), (28, 128, 1), (28, 256, 2), (14, 256, 1), (14, 512, 2), (7, 512, 1)]:
        ho = (hw + 2 - 3) // st + 1
        x = torch.randn(a.batch, c, hw, hw, device=dev).to(bf).contiguous(memory_format=cl)
        gy = torch.randn(a.batch, c, ho, ho, device=dev).to(bf).contiguous(memory_format=cl)
        w4 = torch.randn(c, c, 3, 3, device=dev).to(bf).contiguous(memory_format=cl)
        us_o = timeit(lambda: _C.conv_wgrad(gy, x, 3, 3, st, 1), a.iters)
        us_m = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w4, None, (st, st), (1, 1), (1, 1), False,
                                                                  (0, 0), 1, (False, True, False)), a.iters)
        us_d = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w4, None, (st, st), (1, 1), (1, 1), False,
                                                                  (0, 0), 1, (True, False, False)), a.iters)
        us_f = timeit(lambda: F.conv2d(x, w4, None, st, 1), a.iters)
        wf = w4.permute(0, 2, 3, 1).contiguous()
        wd = w4.flip(2, 3).permute(1, 2, 3, 0).contiguous()
        us_of = timeit(lambda: _C.conv_fwd(x, wf, 3, 3, st, 1, True), a.iters)
        if st == 1:
            us_od = timeit(lambda: _C.conv_fwd(gy, wd, 3, 3, 1, 1, False), a.iters)
        else:
            from distributed_compute_pytorch_amd.ops.conv import _parity_weights
            subs = _parity_weights(wd)
            us_od = timeit(lambda: _C.conv_dgrad_s2(gy, subs, hw, hw), a.iters)
        flops = 2.0 * a.batch * ho * ho * c * c * 9
        r3 = {"shape3x3": f"{hw}x{hw} c={c} s={st}", "ours_wgrad_us": round(us_o, 1), "miopen_wgrad_us": round(us_m, 1),
              "miopen_dgrad_us": round(us_d, 1), "miopen_fwd_us": round(us_f, 1),
              "ours_fwd+stats_us": round(us_of, 1), "ours_dgrad_us": round(us_od, 1),
              "ours_fwd_TFps": round(flops / (us_of * 1e-6) / 1e12, 1),
              "ours_wgrad_TFps": round(flops / (us_o * 1e-6) / 1e12, 1)}
        print(json.dumps(r3), flush=True)
        rows3 = locals().setdefault("rows3", [])
        rows3.append(r3)
    tot = {k: round(sum(r[k] for r in rows), 1) for k in rows[0] if k.endswith("_us")} if rows else {}
    print(json.dumps({"total_us": tot}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "total_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
