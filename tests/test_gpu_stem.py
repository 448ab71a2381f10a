"""Fused ResNet stem (ops/stem.py, csrc/kernels/stem.hip + the stem GEMM)
against a PyTorch fp32 reference of the same op sequence: conv 7x7/2 on the
bf16-rounded image / weight (output rounded to bf16, as the GEMM stores it),
BatchNorm2d training (batch statistics + running-stat update), ReLU,
max_pool2d 3x3/2/1 — forward values, running statistics, and every gradient
(conv weight, gamma, beta) for a given upstream gradient."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

pytestmark = pytest.mark.gpu


def _reference(x, w, gamma, beta, rm, rv, gp, momentum=0.1, eps=1e-5):
    xb = x.to(torch.bfloat16).float()
    wb = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    y = F.conv2d(xb, wb, stride=2, padding=3)
    # the kernels see the bf16-rounded conv output (straight-through for the grad)
    yq = y + (y.to(torch.bfloat16).float() - y).detach()
    g = gamma.detach().clone().requires_grad_(True)
    b = beta.detach().clone().requires_grad_(True)
    z = F.batch_norm(yq, rm, rv, g, b, training=True, momentum=momentum, eps=eps)
    out = F.max_pool2d(F.relu(z), 3, 2, 1)
    out.backward(gp.float())
    return out.detach(), wb.grad, g.grad, b.grad


@pytest.mark.parametrize("shape", [(4, 64, 64), (2, 224, 224), (3, 48, 80)])
@pytest.mark.parametrize("channels_last", [False, True])
def test_stem_matches_reference(cuda, shape, channels_last):
    from distributed_compute_pytorch_amd.ops.stem import fused_stem

    N, H, W = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(cuda)
    bn = nn.BatchNorm2d(64).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    x = torch.randn(N, 3, H, W, device=cuda)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
        conv = conv.to(memory_format=torch.channels_last)
    OH, OW = (H // 2 - 1) // 2 + 1, (W // 2 - 1) // 2 + 1
    gp = torch.randn(N, 64, OH, OW, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    ref_out, ref_dw, ref_dg, ref_db = _reference(x, conv.weight, bn.weight, bn.bias, rm, rv, gp)

    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = fused_stem(x, conv, bn)
    assert out.dtype == torch.bfloat16 and out.is_contiguous(memory_format=torch.channels_last)
    out.backward(gp)
    torch.cuda.synchronize()
    # bf16 output: ~2^-8 relative; occasional arg-max ties between bf16-equal
    # window values move a gradient to a neighbour -> compare norms there
    torch.testing.assert_close(out.float(), ref_out, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn.running_mean, rm, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, rv, rtol=1e-3, atol=1e-4)
    assert int(bn.num_batches_tracked) == 1

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))

    assert rel(bn.bias.grad, ref_db) < 2e-2, rel(bn.bias.grad, ref_db)
    assert rel(bn.weight.grad, ref_dg) < 3e-2, rel(bn.weight.grad, ref_dg)
    assert rel(conv.weight.grad, ref_dw) < 3e-2, rel(conv.weight.grad, ref_dw)
    assert conv.weight.grad.dtype == torch.float32


def test_stem_dual_output_sums_gradients(cuda):
    from distributed_compute_pytorch_amd.ops.stem import fused_stem

    torch.manual_seed(1)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(cuda)
    bn = nn.BatchNorm2d(64).to(cuda)
    x = torch.randn(2, 3, 32, 32, device=cuda)
    g1 = torch.randn(2, 64, 8, 8, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g2 = torch.randn(2, 64, 8, 8, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a, b = fused_stem(x, conv, bn, dual=True)
    torch.autograd.backward([a, b], [g1, g2])
    dw_dual, dg_dual = conv.weight.grad.clone(), bn.weight.grad.clone()
    conv.weight.grad = None
    bn.weight.grad = None
    bn.bias.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        c = fused_stem(x, conv, bn)
    c.backward((g1.float() + g2.float()).to(torch.bfloat16))
    # the dual path sums g1 + g2 in fp32 inside the kernels; the reference sum is
    # rounded to bf16 first: compare as relative norms
    for got, ref in ((conv.weight.grad, dw_dual), (bn.weight.grad, dg_dual)):
        assert float((got - ref).norm() / ref.norm()) < 2e-2


def test_resnet_uses_fused_stem_and_tracks_module_path(cuda, monkeypatch):
    """ResNet-50-family model: the fused stem is taken under bf16 autocast and the
    loss matches the per-module path (DCP_STEM=0) within bf16 noise."""
    import distributed_compute_pytorch_amd.models.resnet as R

    torch.manual_seed(0)
    m = R.resnet18_like(num_classes=10, fused_bn=True).to(cuda).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device=cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    import distributed_compute_pytorch_amd.ops.stem as S

    calls = {"n": 0}
    orig = S._StemFn.apply

    def counting(*a):
        calls["n"] += 1
        return orig(*a)

    monkeypatch.setattr(S._StemFn, "apply", counting)
    losses = []
    for fused in (True, False):
        monkeypatch.setattr(R, "FUSED_STEM", fused)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            losses.append(float(F.cross_entropy(m(x), y)))
    assert calls["n"] == 1
    assert abs(losses[0] - losses[1]) < 0.03 * max(1.0, abs(losses[1])), losses


@pytest.mark.parametrize("wide", [1, 0])
@pytest.mark.parametrize("shape", [(4, 64, 64), (3, 48, 80), (16, 224, 224)])
def test_stem_conv_wgrad_matches_fp64(cuda, shape, wide):
    """The stem weight-gradient GEMM alone (one 64 x 256 tile per slab, or the
    two 64 x 128 tiles with wide = 0) against an fp64 conv2d weight gradient of
    the same bf16 image and output gradient."""
    from distributed_compute_pytorch_amd._ext import C

    N, H, W = shape
    torch.manual_seed(1)
    x = torch.randn(N, 3, H, W, device=cuda).to(torch.bfloat16)
    dy = torch.randn(N, 64, H // 2, W // 2, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    old = C.gemm_tune_get("stem_wide")
    try:
        C.gemm_tune("stem_wide", wide)
        xp, _ = C.stem_prep(x, False)
        dw = C.stem_conv_wgrad(dy, xp, H, W)
        torch.cuda.synchronize()
    finally:
        C.gemm_tune("stem_wide", old)
    ref = torch.nn.grad.conv2d_weight(x.double().cpu(), (64, 3, 7, 7), dy.double().cpu(), stride=2, padding=3)
    err = (dw.double().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert dw.dtype == torch.float32 and dw.shape == (64, 3, 7, 7)
    assert err <= 1e-4 * scale + 1e-3, (err, scale)
