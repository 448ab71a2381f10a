"""Isolate fp32 gradient differences between the stock and fused ResNet-50.

Prints, per variant, the relative gradient error of a few parameters against
the stock ATen model (and stock-vs-stock to show MIOpen's own run-to-run noise).
"""
import torch
import torch.nn.functional as F

from distributed_compute_pytorch_amd.models import resnet50

dev = torch.device("cuda", 0)
torch.manual_seed(0)
ref = resnet50(num_classes=100).to(dev).to(memory_format=torch.channels_last)
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(16, 3, 96, 96, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 100, (16,), generator=g).to(dev)


def grads(m):
    m.zero_grad(set_to_none=True)
    F.cross_entropy(m(x), y).backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


base = grads(ref)
names = ["conv1.weight", "bn1.weight", "layer1.0.conv1.weight", "layer2.0.conv1.weight", "layer3.0.conv2.weight",
         "layer4.2.conv3.weight", "layer4.2.bn3.weight", "fc.weight"]
variants = {
    "stock again": dict(),
    "fused bn+pool+dual": dict(fused_bn=True),
    "fused bn, stock pool, dual": dict(fused_bn=True, fused_pool=False),
    "fused bn+pool, no dual": dict(fused_bn=True, dual_bn=False),
    "fused bn, stock pool, no dual": dict(fused_bn=True, fused_pool=False, dual_bn=False),
    "stock bn, fused pool": dict(fused_pool=True),
}
for name, kw in variants.items():
    m = resnet50(num_classes=100, **kw).to(dev).to(memory_format=torch.channels_last)
    m.load_state_dict(ref.state_dict())
    gr = grads(m)
    errs = {n: float((gr[n] - base[n]).norm() / base[n].norm().clamp_min(1e-12)) for n in names}
    worst = max(((float((gr[n] - base[n]).norm() / base[n].norm().clamp_min(1e-12)), n) for n in base))
    print(f"{name:34s} worst={worst[0]:.2e} ({worst[1]}) " + " ".join(f"{k.split('.')[0]}:{v:.1e}" for k, v in errs.items()),
          flush=True)
