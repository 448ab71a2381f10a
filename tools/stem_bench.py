"""ResNet-50 stem conv (7x7/2, 3->64) on MIOpen NHWC bf16: channel padding 3 -> 4 / 8.
Forward + weight-grad only (the input needs no grad), batch 256."""
import json
import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")


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


B = 256
x3 = torch.randn(B, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
w3 = torch.randn(64, 3, 7, 7, device=dev, dtype=torch.float32, requires_grad=True)
for cpad in (3, 4, 8):
    def fb():
        if cpad == 3:
            x, w = x3, w3.to(torch.bfloat16)
        else:
            x = torch.zeros(B, cpad, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            x[:, :3] = x3
            w = F.pad(w3, (0, 0, 0, 0, 0, cpad - 3)).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=2, padding=3)
        y.backward(torch.ones_like(y))
    print(json.dumps({"cpad": cpad, "ms_fwd_wgrad_incl_pad": round(timeit(fb), 4)}), flush=True)
