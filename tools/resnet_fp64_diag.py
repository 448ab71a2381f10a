"""Per-parameter gradient error of one fp32 ResNet-50 step against an fp64 CPU
reference of the same model, input and labels: stock ATen/MIOpen fp32 on the
GPU vs our fused-BN DDP model. Prints the worst parameters (rel L2 error).

    python tools/resnet_fp64_diag.py [--tf32 0|1]

--tf32 0 turns off the reduced-precision fp32 convolutions / matmuls
(torch.backends.cudnn.allow_tf32 defaults to True: MIOpen may then run fp32
convolutions in xf32). Also prints the forward activations of the last
bottleneck's modules against the fp64 reference (relative L2).
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port
    from distributed_compute_pytorch_amd.models import resnet50

    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--tf32", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.allow_tf32 = bool(a.tf32)
    torch.backends.cuda.matmul.allow_tf32 = bool(a.tf32)
    print(f"allow_tf32 = {bool(a.tf32)}")
    cuda = torch.device("cuda", 0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    torch.manual_seed(0)
    cpu = resnet50(num_classes=100)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(16, 3, 96, 96, generator=g)
    y = torch.randint(0, 100, (16,), generator=g)
    ref = copy.deepcopy(cpu).double()
    acts = {}

    def hook(tag):
        def h(name):
            def f(mod, inp, out):
                o = out[0] if isinstance(out, tuple) else out
                if isinstance(o, torch.Tensor):
                    acts.setdefault(name, {})[tag] = o.detach().double().cpu()
            return f
        return h

    def watch(model, tag):
        for name, mod in model.named_modules():
            if name.startswith(("layer4.2.", "layer4.1.", "layer1.0.")) or name in ("conv1", "bn1", "fc"):
                mod.register_forward_hook(hook(tag)(name))

    watch(ref, "ref")
    F.cross_entropy(ref(x.double()), y).backward()
    g64 = {n: p.grad for n, p in ref.named_parameters()}
    c32 = copy.deepcopy(cpu)
    F.cross_entropy(c32(x), y).backward()  # fp32 on the CPU: the conditioning of the problem itself
    g32 = {n: p.grad for n, p in c32.named_parameters()}
    stock = copy.deepcopy(cpu).to(cuda).to(memory_format=torch.channels_last)
    ours_m = resnet50(num_classes=100, fused_bn=True)
    ours_m.load_state_dict(cpu.state_dict())
    ours_m = ours_m.to(cuda).to(memory_format=torch.channels_last)
    ddp = dcp.parallel.DistributedDataParallel(ours_m, device_ids=[0], gradient_as_bucket_view=True)
    xc = x.to(cuda).contiguous(memory_format=torch.channels_last)
    watch(stock, "stock")
    watch(ours_m, "ours")
    F.cross_entropy(stock(xc), y.to(cuda)).backward()
    F.cross_entropy(ddp(xc), y.to(cuda)).backward()
    print("forward activations, rel L2 vs fp64:  module  stock  ours")
    for name, d in acts.items():
        if "ref" in d:
            r = d["ref"]
            e = {t: float((d[t].reshape(r.shape) - r).norm() / r.norm().clamp_min(1e-30)) for t in ("stock", "ours")
                 if t in d and d[t].numel() == r.numel()}
            print(f"  {name:32s} " + " ".join(f"{t}={v:.2e}" for t, v in e.items()))
    rows = []
    for (n, ps), po in zip(stock.named_parameters(), ours_m.parameters()):
        r = g64[n]
        den = r.norm().clamp_min(1e-30)
        rows.append((n, float((ps.grad.double().cpu() - r).norm() / den), float((po.grad.double().cpu() - r).norm() / den),
                     float((g32[n].double() - r).norm() / den)))
    rows.sort(key=lambda t: -t[2] / max(t[3], 1e-12))
    print("param  stock_gpu_fp32_vs_fp64  ours_vs_fp64  cpu_fp32_vs_fp64")
    for n, a, b, c in rows[:25]:
        print(f"{n:40s} {a:.3e} {b:.3e} {c:.3e}")
    import statistics
    ratios = sorted(r[2] / max(r[3], 1e-12) for r in rows)
    print("ours/cpu32 ratio: median", statistics.median(ratios), "p90", ratios[int(0.9 * len(ratios))], "max",
          ratios[-1], "| stock/cpu32 median", statistics.median(r[1] / max(r[3], 1e-12) for r in rows))
    print("max stock", max(r[1] for r in rows), "max ours", max(r[2] for r in rows), "max cpu fp32",
          max(r[3] for r in rows))
    dcp.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
