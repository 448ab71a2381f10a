"""Microbenchmark: ResNet-50 convolutions (bf16, channels_last) via MIOpen vs
1x1-as-GEMM (hipBLASLt) — forward + backward (dgrad + wgrad), batch 256."""
import json
import sys

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
# (Cin, Cout, k, stride, H_in)
SHAPES = [
    (3, 64, 7, 2, 224),
    (64, 64, 1, 1, 56), (64, 64, 3, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56), (64, 256, 1, 1, 56),
    (256, 128, 1, 1, 56), (128, 128, 3, 2, 56), (128, 512, 1, 1, 28), (256, 512, 1, 2, 56),
    (512, 128, 1, 1, 28), (128, 128, 3, 1, 28),
    (512, 256, 1, 1, 28), (256, 256, 3, 2, 28), (256, 1024, 1, 1, 14), (512, 1024, 1, 2, 28),
    (1024, 256, 1, 1, 14), (256, 256, 3, 1, 14),
    (1024, 512, 1, 1, 14), (512, 512, 3, 2, 14), (512, 2048, 1, 1, 7), (1024, 2048, 1, 2, 14),
    (2048, 512, 1, 1, 7), (512, 512, 3, 1, 7),
]


def timeit(fn, n=20, w=5):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


res = []
for cin, cout, k, st, h in SHAPES:
    x = torch.randn(B, cin, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    w.requires_grad_()
    y = F.conv2d(x, w, stride=st, padding=k // 2)
    gy = torch.randn_like(y)
    ho = y.shape[2]
    flop = 2 * B * ho * ho * cout * cin * k * k

    def conv_fb():
        out = F.conv2d(x, w, stride=st, padding=k // 2)
        gx, gw = torch.autograd.grad(out, (x, w), gy)

    t_conv = timeit(conv_fb)
    t_gemm = None
    if k == 1:
        def gemm_fb():
            xx = x if st == 1 else x[:, :, ::st, ::st]
            a = xx.permute(0, 2, 3, 1).reshape(-1, cin)
            out = F.linear(a, w.view(cout, cin))
            gx, gw = torch.autograd.grad(out, (x, w), gy.permute(0, 2, 3, 1).reshape(-1, cout))

        t_gemm = timeit(gemm_fb)
    r = dict(cin=cin, cout=cout, k=k, stride=st, h=h, conv_ms=round(t_conv, 4),
             gemm_ms=None if t_gemm is None else round(t_gemm, 4), conv_tflops=round(3 * flop / t_conv / 1e9, 1),
             gemm_tflops=None if t_gemm is None else round(3 * flop / t_gemm / 1e9, 1))
    res.append(r)
    print(json.dumps(r), flush=True)
tot_conv = sum(r["conv_ms"] for r in res)
tot_best = sum(min(r["conv_ms"], r["gemm_ms"] or 1e9) for r in res)
print(json.dumps({"sum_conv_ms": round(tot_conv, 3), "sum_best_ms": round(tot_best, 3)}))
