"""Accuracy of the fused BatchNorm(+ReLU)(+residual) forward/backward in fp32
against an fp64 ATen oracle, next to stock fp32 ATen: rel L2 error of y, dx,
dgamma, dbeta (and dres) per shape. Also prints the device's CU count.

    python tools/bn_fp64_probe.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d

    dev = torch.device("cuda", 0)
    p = torch.cuda.get_device_properties(0)
    print("device", p.name, "CUs", p.multi_processor_count, flush=True)
    g = torch.Generator().manual_seed(0)
    for (n, c, h, w) in [(16, 2048, 3, 3), (16, 512, 3, 3), (16, 256, 6, 6), (16, 64, 24, 24)]:
        for act, res in ((True, False), (False, False), (True, True)):
            x = (torch.randn(n, c, h, w, generator=g) * 3 + 1).to(dev).contiguous(memory_format=torch.channels_last)
            r = torch.randn(n, c, h, w, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
            dy = torch.randn(n, c, h, w, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
            gam = torch.rand(c, generator=g).to(dev) + 0.5
            bet = torch.randn(c, generator=g).to(dev)
            out = {}
            for arm in ("fused", "stock", "fp64"):
                dt = torch.float64 if arm == "fp64" else torch.float32
                bn = BatchNormAct2d(c, act=act, residual=res, fused=arm == "fused").to(dev).to(dt)
                with torch.no_grad():
                    bn.weight.copy_(gam)
                    bn.bias.copy_(bet)
                xi = x.to(dt).detach().requires_grad_(True)
                ri = r.to(dt).detach().requires_grad_(True)
                y = bn(xi, ri) if res else bn(xi)
                y.backward(dy.to(dt))
                out[arm] = (y.detach(), xi.grad, bn.weight.grad, bn.bias.grad, ri.grad if res else None)
            names = ("y", "dx", "dgamma", "dbeta", "dres")
            line = []
            for i, nm in enumerate(names):
                if out["fp64"][i] is None:
                    continue
                line.append(f"{nm} fused {rel(out['fused'][i], out['fp64'][i]):.1e} stock "
                            f"{rel(out['stock'][i], out['fp64'][i]):.1e}")
            print(f"[{n},{c},{h},{w}] act={int(act)} res={int(res)}: " + "; ".join(line), flush=True)


if __name__ == "__main__":
    main()
