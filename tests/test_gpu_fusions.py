"""Round-2 ResNet fusions against PyTorch fp32 references:

* relu(bn3(x) + bn_ds(x2)) with the downsample BatchNorm applied inside BN3's
  residual kernel (ops/batchnorm.py bn_resbn_act): outputs, both sets of
  running statistics, and every gradient (x, x2, both gammas / betas), with a
  dual-output (two consumers) upstream gradient;
* ConvWeightPrep: every conv's bf16 GEMM operands from one launch are
  bit-identical to the per-conv cast kernels, and a ResNet step with it equals
  the step without it.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _sums(x):
    xf = x.float().permute(0, 2, 3, 1).reshape(-1, x.shape[1])
    return torch.cat([xf.sum(0), (xf * xf).sum(0)]).contiguous()


@pytest.mark.parametrize("C,hw", [(256, 14), (512, 7), (64, 8)])
def test_resbn_matches_reference(cuda, C, hw):
    from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d, bn_resbn_act

    torch.manual_seed(0)
    N = 6
    bn3 = BatchNormAct2d(C, act=True, residual=True, fused=True).to(cuda)
    bnd = BatchNormAct2d(C, act=False, fused=True).to(cuda)
    with torch.no_grad():
        for m in (bn3, bnd):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.5, 0.5)
            m.running_mean.uniform_(-0.1, 0.1)
    ref3, refd = copy.deepcopy(bn3), copy.deepcopy(bnd)
    cl = torch.channels_last
    x = (torch.randn(N, C, hw, hw, device=cuda) * 2 + 0.3).to(torch.bfloat16).contiguous(memory_format=cl)
    x2 = (torch.randn(N, C, hw, hw, device=cuda) * 0.7 - 0.2).to(torch.bfloat16).contiguous(memory_format=cl)
    gy = torch.randn(N, C, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)
    gy2 = torch.randn(N, C, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)

    xa = x.detach().clone().requires_grad_(True)
    x2a = x2.detach().clone().requires_grad_(True)
    y, ya = bn_resbn_act(bn3, xa, _sums(x), bnd, x2a, _sums(x2), dual=True)
    torch.autograd.backward([y, ya], [gy, gy2])

    xr = x.float().requires_grad_(True)
    x2r = x2.float().requires_grad_(True)
    yr = F.relu(F.batch_norm(xr, ref3.running_mean, ref3.running_var, ref3.weight, ref3.bias, True, 0.1, 1e-5)
                + F.batch_norm(x2r, refd.running_mean, refd.running_var, refd.weight, refd.bias, True, 0.1, 1e-5))
    yr.backward(gy.float() + gy2.float())

    torch.testing.assert_close(y.float(), yr.detach(), rtol=2e-2, atol=2e-2)
    for a, b in ((bn3, ref3), (bnd, refd)):
        torch.testing.assert_close(a.running_mean, b.running_mean, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(a.running_var, b.running_var, rtol=1e-4, atol=1e-5)
        assert int(a.num_batches_tracked) == 1

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))

    assert rel(xa.grad, xr.grad) < 2e-2
    assert rel(x2a.grad, x2r.grad) < 2e-2
    for a, b in ((bn3, ref3), (bnd, refd)):
        assert rel(a.weight.grad, b.weight.grad) < 2e-2, (rel(a.weight.grad, b.weight.grad))
        assert rel(a.bias.grad, b.bias.grad) < 2e-2


def test_weight_prep_matches_per_conv_casts(cuda):
    from distributed_compute_pytorch_amd._ext import C as _C
    from distributed_compute_pytorch_amd.ops.conv import ConvWeightPrep

    torch.manual_seed(0)
    shapes = [(64, 64, 1), (256, 64, 1), (128, 128, 3), (512, 256, 1), (64, 64, 3), (2048, 512, 1)]
    ws = [torch.randn(co, ci, k, k, device=cuda).contiguous(memory_format=torch.channels_last)
          for co, ci, k in shapes]
    prep = ConvWeightPrep(ws)
    with prep:
        for w, b, t in zip(ws, prep.wb, prep.wt):
            k = w.shape[2]
            if k == 1:
                rb, rt = _C.weight_bf16_t(w)
                assert torch.equal(b.view(b.shape[0], -1), rb) and torch.equal(t.view(t.shape[0], -1), rt)
            else:
                rb, rt = _C.conv_weight_bf16(w)
                assert torch.equal(b, rb) and torch.equal(t, rt)


def test_resnet_step_with_prep_and_resbn_matches_plain(cuda, monkeypatch):
    """One bf16 training step of a small bottleneck ResNet: the round-2 paths
    (ConvWeightPrep, fused residual BN, fused stem) give the same loss and
    gradients as the per-op paths within bf16 noise."""
    import distributed_compute_pytorch_amd.models.resnet as R

    torch.manual_seed(0)
    base = R.resnet18_like(num_classes=10, fused_bn=True).to(cuda).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    res = []
    for on in (True, False, False):  # the plain path twice: its own run-to-run spread is the noise floor
        monkeypatch.setattr(R, "WEIGHT_PREP", on)
        monkeypatch.setattr(R, "RESBN", on)
        monkeypatch.setattr(R, "FUSED_STEM", on)
        m = copy.deepcopy(base)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        res.append((float(loss), torch.cat([p.grad.float().reshape(-1) for p in m.parameters()]),
                    torch.cat([b.float().reshape(-1) for b in m.buffers()])))
    (l1, g1, b1), (l2, g2, b2), (_, g3, _) = res
    assert abs(l1 - l2) < 1e-2 * max(1.0, abs(l2)), (l1, l2)
    # a random-init bf16 bottleneck net at batch 8 amplifies rounding-order noise
    # (atomic BN sums, MIOpen) into 10-20 % on BN-bias gradients between two
    # identical runs; a wrong kernel gives O(1) or non-finite differences
    err = float((g1 - g2).norm() / g2.norm())
    noise = float((g3 - g2).norm() / g2.norm())
    assert bool(torch.isfinite(g1).all())
    assert err < 4 * noise + 0.05, (err, noise)
    torch.testing.assert_close(b1, b2, rtol=2e-2, atol=2e-2)
