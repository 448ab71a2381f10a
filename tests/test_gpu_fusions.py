"""Round-2 ResNet fusions against PyTorch fp32 references:

* relu(bn3(x) + bn_ds(x2)) with the downsample BatchNorm applied inside BN3's
  residual kernel (ops/batchnorm.py bn_resbn_act): outputs, both sets of
  running statistics, and every gradient (x, x2, both gammas / betas), with a
  dual-output (two consumers) upstream gradient;
* the block-boundary node relu(bn3(z3) + r) → next conv1 with BN3's backward
  reduction in the conv1 data-gradient epilogue (ops/conv.py bn_res_act_conv1x1);
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


@pytest.mark.parametrize("C,Co,N,hw,resbn,with_gy", [(256, 64, 4, 14, False, True), (256, 64, 4, 14, True, True),
                                                     (512, 128, 3, 9, False, True), (1024, 256, 2, 7, True, True),
                                                     (256, 64, 4, 14, False, False)])
def test_bn_res_act_conv1x1_matches_reference(cuda, C, Co, N, hw, resbn, with_gy):
    """Block boundary node (ops/conv.py bn_res_act_conv1x1): relu(bn3(z3) + r)
    → next conv1, with BN3's backward reduced in conv1's dgrad epilogue
    (gemm.hip RESRED), against the fp32 composition: outputs, sums, running
    statistics and every gradient. M = N·hw² is ragged for hw = 9, 7."""
    from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d
    from distributed_compute_pytorch_amd.ops.conv import bn_res_act_conv1x1

    torch.manual_seed(1)
    cl = torch.channels_last
    bn3 = BatchNormAct2d(C, act=True, residual=True, fused=True).to(cuda)
    bnd = BatchNormAct2d(C, act=False, fused=True).to(cuda)
    with torch.no_grad():
        for m in (bn3, bnd):
            m.weight.uniform_(0.5, 1.5)
            m.bias.uniform_(-0.5, 0.5)
    ref3, refd = copy.deepcopy(bn3), copy.deepcopy(bnd)
    w = (torch.randn(Co, C, 1, 1, device=cuda) / C ** 0.5).contiguous(memory_format=cl).requires_grad_(True)
    z3 = (torch.randn(N, C, hw, hw, device=cuda) * 1.5 + 0.2).to(torch.bfloat16).contiguous(memory_format=cl)
    r = (torch.randn(N, C, hw, hw, device=cuda) * 0.8).to(torch.bfloat16).contiguous(memory_format=cl)
    gy = torch.randn(N, C, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)
    gz = torch.randn(N, Co, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)

    za = z3.detach().clone().requires_grad_(True)
    ra = r.detach().clone().requires_grad_(True)
    if resbn:
        y, z1, s1 = bn_res_act_conv1x1(bn3, za, _sums(z3), None, w, (bnd, ra, _sums(r)))
    else:
        y, z1, s1 = bn_res_act_conv1x1(bn3, za, _sums(z3), ra, w)
    if with_gy:
        torch.autograd.backward([y, z1], [gy, gz])
    else:  # y's own consumer unused: no second gradient (RESRED's gy2 = None path)
        z1.backward(gz)
        gy = torch.zeros_like(gy)

    zr = z3.float().requires_grad_(True)
    rr = r.float().requires_grad_(True)
    wr = w.detach().float().clone().requires_grad_(True)
    res = (F.batch_norm(rr, refd.running_mean, refd.running_var, refd.weight, refd.bias, True, 0.1, 1e-5)
           if resbn else rr)
    yr = F.relu(F.batch_norm(zr, ref3.running_mean, ref3.running_var, ref3.weight, ref3.bias, True, 0.1, 1e-5)
                + res)
    z1r = F.conv2d(yr, wr)
    torch.autograd.backward([yr, z1r], [gy.float(), gz.float()])

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))

    assert rel(y, yr) < 1e-2
    assert rel(z1, z1r) < 2e-2
    torch.testing.assert_close(s1, _sums(z1), rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(bn3.running_mean, ref3.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn3.running_var, ref3.running_var, rtol=1e-4, atol=1e-5)
    assert rel(za.grad, zr.grad) < 3e-2, rel(za.grad, zr.grad)
    assert rel(ra.grad, rr.grad) < 3e-2, rel(ra.grad, rr.grad)
    assert rel(w.grad, wr.grad) < 2e-2
    pairs = [(bn3, ref3)] + ([(bnd, refd)] if resbn else [])
    for a, b in pairs:
        assert rel(a.weight.grad, b.weight.grad) < 3e-2, rel(a.weight.grad, b.weight.grad)
        assert rel(a.bias.grad, b.bias.grad) < 3e-2, rel(a.bias.grad, b.bias.grad)


def test_resnet_step_chain_fusion_matches_unfused(cuda, monkeypatch):
    """A bf16 training step of a small bottleneck ResNet with every BN3 fused
    into the next block's conv1 node (DCP_RES_CONV_FUSE) equals the unfused
    chain within the run-to-run noise floor."""
    import distributed_compute_pytorch_amd.models.resnet as R

    torch.manual_seed(0)
    base = R.ResNet(R.Bottleneck, [2, 2, 1, 1], num_classes=10, fused_bn=True).to(cuda).to(
        memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    res = []
    for on in (True, False, False):
        monkeypatch.setattr(R, "RES_CONV_FUSE", on)
        m = copy.deepcopy(base)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        res.append((float(loss), torch.cat([p.grad.float().reshape(-1) for p in m.parameters()]),
                    torch.cat([b.float().reshape(-1) for b in m.buffers()])))
    (l1, g1, b1), (l2, g2, b2), (_, g3, _) = res
    assert abs(l1 - l2) < 1e-2 * max(1.0, abs(l2)), (l1, l2)
    err = float((g1 - g2).norm() / g2.norm())
    noise = float((g3 - g2).norm() / g2.norm())
    assert bool(torch.isfinite(g1).all())
    assert err < 4 * noise + 0.05, (err, noise)
    torch.testing.assert_close(b1, b2, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("C,Co,N,hw", [(256, 64, 4, 14), (512, 128, 3, 9), (1024, 256, 2, 7), (256, 64, 2, 56)])
def test_res_prologue_matches_apply_pass(cuda, C, Co, N, hw):
    """The identity block boundary with BN3 + residual + ReLU as conv1's GEMM
    prologue (gemm.hip RES, ops/conv.py RES_PROLOGUE) against the separate
    apply pass + plain GEMM: y and its ReLU mask bit-identical (same fp32
    expression), z1 / sums / running statistics / every gradient matching.
    Covers 64- and 128-column tiles, one and two N-tiles, 128- and 256-row
    tiles and ragged row counts (M = N·hw²)."""
    from distributed_compute_pytorch_amd.ops import conv as conv_ops
    from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d

    torch.manual_seed(3)
    cl = torch.channels_last
    z3 = (torch.randn(N, C, hw, hw, device=cuda) * 1.5 + 0.2).to(torch.bfloat16).contiguous(memory_format=cl)
    r = (torch.randn(N, C, hw, hw, device=cuda) * 0.8).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(Co, C, 1, 1, device=cuda) / C ** 0.5).contiguous(memory_format=cl)
    gy = torch.randn(N, C, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)
    gz = torch.randn(N, Co, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=cl)
    outs = {}
    for on in (False, True):
        conv_ops.RES_PROLOGUE = on
        try:
            bn = BatchNormAct2d(C, act=True, residual=True, fused=True).to(cuda)
            with torch.no_grad():
                bn.weight.copy_(torch.linspace(0.5, 1.5, C))
                bn.bias.copy_(torch.linspace(-0.5, 0.5, C))
            za, ra = z3.clone().requires_grad_(True), r.clone().requires_grad_(True)
            wa = w.clone().requires_grad_(True)
            y, z1, s1 = conv_ops.bn_res_act_conv1x1(bn, za, _sums(z3), ra, wa)
            torch.autograd.backward([y, z1], [gy, gz])
            outs[on] = (y.detach(), z1.detach(), s1, bn.running_mean.clone(), bn.running_var.clone(), za.grad,
                        ra.grad, wa.grad, bn.weight.grad, bn.bias.grad)
        finally:
            conv_ops.RES_PROLOGUE = False
    a, b = outs[False], outs[True]
    assert torch.equal(a[0], b[0])  # y: same expression, same rounding

    def rel(x, y_):
        return float((x.float() - y_.float()).norm() / y_.float().norm().clamp_min(1e-12))

    assert rel(b[1], a[1]) < 1e-2  # z1: same operands, another k order (BK 32 vs 64)
    torch.testing.assert_close(b[2], a[2], rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(b[3], a[3], rtol=0, atol=0)
    torch.testing.assert_close(b[4], a[4], rtol=0, atol=0)
    for i in range(5, 10):
        assert rel(b[i], a[i]) < 1e-2, (i, rel(b[i], a[i]))
