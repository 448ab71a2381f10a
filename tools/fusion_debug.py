"""Per-parameter gradient differences of a small bottleneck ResNet bf16 step
under the round-2 fusion toggles (WEIGHT_PREP, RESBN, FUSED_STEM) against the
all-off path, with an all-off repeat as the noise floor."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_compute_pytorch_amd.models.resnet as R  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
base = R.resnet18_like(num_classes=10, fused_bn=True).to(dev).to(memory_format=torch.channels_last)
x = torch.randn(8, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (8,), device=dev)


def run(prep, resbn, stem):
    R.WEIGHT_PREP, R.RESBN, R.FUSED_STEM = prep, resbn, stem
    m = copy.deepcopy(base)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()}


ref_l, ref = run(False, False, False)
for cfg in [(False, False, False), (True, False, False), (False, True, False), (False, False, True),
            (True, True, True)]:
    l, g = run(*cfg)
    worst = sorted(((float((g[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-12)), n) for n in ref), reverse=True)
    print(f"prep={cfg[0]} resbn={cfg[1]} stem={cfg[2]} loss {l:.5f} vs {ref_l:.5f}; worst:",
          ", ".join(f"{n}={v:.3f}" for v, n in worst[:6]), flush=True)
