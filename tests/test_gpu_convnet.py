"""Fused ConvNet path (reference model, main.py:20-45): BN1d+ReLU, fused
relu+maxpool+Dropout2d, log-softmax — each against the fp32 ATen composition."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn1d_relu_matches_aten(cuda, dtype):
    from distributed_compute_pytorch_amd.ops import BatchNormAct1d

    torch.manual_seed(0)
    ref = torch.nn.BatchNorm1d(128).to(cuda)
    ours = BatchNormAct1d(128, act=True, fused=True).to(cuda)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.normal_()
    ours.load_state_dict(ref.state_dict())
    x = torch.randn(128, 128, device=cuda) * 3 + 1
    xr = x.clone().requires_grad_()
    xo = x.to(dtype).requires_grad_()
    yr = F.relu(ref(xr))
    yo = ours(xo)
    g = torch.randn_like(yr)
    yr.backward(g)
    yo.backward(g.to(dtype))
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(yo.float(), yr, **tol)
    torch.testing.assert_close(ours.running_mean, ref.running_mean, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(ours.running_var, ref.running_var, rtol=1e-3, atol=1e-3)
    assert int(ours.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    rel = lambda a, b: float((a.float() - b).norm() / b.norm())
    lim = 1e-4 if dtype == torch.float32 else 2e-2
    assert rel(xo.grad, xr.grad) < lim
    assert rel(ours.weight.grad, ref.weight.grad) < lim
    assert rel(ours.bias.grad, ref.bias.grad) < lim


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(128, 10), (64, 1000), (7, 3)])
def test_log_softmax_matches_aten(cuda, dtype, shape):
    from distributed_compute_pytorch_amd.ops import fused_log_softmax

    torch.manual_seed(0)
    x = (torch.randn(shape, device=cuda) * 4).to(dtype)
    xr = x.detach().float().clone().requires_grad_()
    xo = x.detach().clone().requires_grad_()
    yr = F.log_softmax(xr, 1)
    yo = fused_log_softmax(xo, 1)
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(yo.float(), yr, **tol)
    g = torch.randn_like(yr)
    yr.backward(g)
    yo.backward(g.to(yo.dtype))
    torch.testing.assert_close(xo.grad.float(), xr.grad, **tol)


def test_log_softmax_autocast_outputs_fp32(cuda):
    from distributed_compute_pytorch_amd.ops import fused_log_softmax

    x = torch.randn(32, 10, device=cuda, dtype=torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = fused_log_softmax(x, 1)
    assert y.dtype == torch.float32
    torch.testing.assert_close(y, F.log_softmax(x.float(), 1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_relu_pool_dropout(cuda, dtype):
    from distributed_compute_pytorch_amd.ops import relu_max_pool2d_dropout

    torch.manual_seed(0)
    x = torch.randn(16, 64, 24, 24, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    # p = 0: exactly relu → maxpool
    xr = x.detach().float().clone().requires_grad_()
    xo = x.detach().clone().requires_grad_()
    yr = F.max_pool2d(F.relu(xr), 2)
    yo = relu_max_pool2d_dropout(xo, 2, 2, 0, 0.0, True)
    torch.testing.assert_close(yo.float(), yr, rtol=0, atol=0)
    g = torch.randn_like(yr)
    yr.backward(g)
    yo.backward(g.to(dtype))
    torch.testing.assert_close(xo.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)
    # p = 0.25: whole (n, c) planes dropped, kept ones scaled by 4/3, and the
    # backward applies the same mask
    xo2 = x.detach().clone().requires_grad_()
    yd = relu_max_pool2d_dropout(xo2, 2, 2, 0, 0.25, True)
    base = F.max_pool2d(F.relu(x.float()), 2)
    nz = base.abs().sum((2, 3)) > 0
    kept = yd.float().abs().sum((2, 3)) > 0
    frac = (kept & nz).sum().item() / nz.sum().item()
    assert 0.65 < frac < 0.85, frac
    scale = torch.where(kept, torch.full_like(base[:, :, 0, 0], 4.0 / 3.0), torch.zeros_like(base[:, :, 0, 0]))
    torch.testing.assert_close(yd.float(), base * scale[:, :, None, None], rtol=1e-2, atol=1e-2)
    yd.backward(torch.ones_like(yd))
    # dropped planes get no gradient
    gsum = xo2.grad.float().abs().sum((2, 3))
    assert bool(((~kept) & nz).logical_and(gsum > 0).sum() == 0)
    assert bool((kept & nz).logical_and(gsum == 0).sum() == 0)


def test_fused_convnet_matches_stock(cuda):
    """Same weights: eval outputs equal; one train step's gradients equal with dropout off."""
    from distributed_compute_pytorch_amd.models import ConvNet

    torch.manual_seed(0)
    ref = ConvNet().to(cuda)
    ours = ConvNet(fused=True).to(cuda)
    ours.load_state_dict(ref.state_dict())
    assert list(ours.state_dict().keys()) == list(ref.state_dict().keys())
    x = torch.randn(64, 1, 28, 28, device=cuda)
    y = torch.randint(0, 10, (64,), device=cuda)
    ref.eval(), ours.eval()
    with torch.no_grad():
        torch.testing.assert_close(ours(x), ref(x), rtol=1e-4, atol=1e-4)
    ref.train(), ours.train()
    for m in (ref, ours):
        m.dropout1.p = 0.0
        m.dropout2.p = 0.0
    F.nll_loss(ref(x), y).backward()
    F.nll_loss(ours(x), y).backward()
    for (n, p), q in zip(ref.named_parameters(), ours.parameters()):
        if n == "fc1.bias":
            # BN right after fc1 cancels any per-channel shift: this gradient is
            # 0 up to rounding noise in both implementations
            assert float(q.grad.abs().max()) < 1e-4 * float(ours.fc1.weight.grad.abs().max()) + 1e-6
            continue
        rel = float((q.grad - p.grad).norm() / p.grad.norm().clamp_min(1e-12))
        assert rel < 1e-3, (n, rel)
    torch.testing.assert_close(ours.batchnorm.running_mean, ref.batchnorm.running_mean, rtol=1e-4, atol=1e-5)


def test_fused_convnet_trains(cuda):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.models import ConvNet

    torch.manual_seed(0)
    m = ConvNet(fused=True).to(cuda)
    opt = dcp.optim.Adadelta(m.parameters(), lr=1.0)
    x = torch.randn(128, 1, 28, 28, device=cuda)
    y = torch.randint(0, 10, (128,), device=cuda)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss = F.nll_loss(m(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses


def _features_ref(x, m, drop_scale=None):
    """fp64 CPU composition (exact up to fp64 rounding): ATen's fp32 GPU convs
    may pick Winograd-type algorithms whose own error is ~1e-3 relative."""
    import copy

    m64 = copy.deepcopy(m).double().cpu()
    y = F.max_pool2d(F.relu(m64.conv2(F.relu(m64.conv1(x.double().cpu())))), 2)
    if drop_scale is not None:
        y = y * drop_scale.double().cpu()[:, :, None, None]
    return torch.flatten(y, 1), m64


def _ref_grads(x, m, g, names, drop_scale=None):
    y, m64 = _features_ref(x, m, drop_scale)
    ps = [dict(m64.named_parameters())[n] for n in names]
    return y, [t.float().to(x.device) for t in torch.autograd.grad(y, ps, g.double().cpu())]


_NAMES = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"]


@pytest.mark.parametrize("B", [128, 5])
def test_convnet_features_kernel_matches_fp32(cuda, B):
    """The fused conv1→ReLU→conv2→ReLU→pool→flatten kernel (fp32 MFMA) and its
    backward against the fp64 composition on the same weights."""
    from distributed_compute_pytorch_amd.models import ConvNet
    from distributed_compute_pytorch_amd.ops import convnet_features

    torch.manual_seed(0)
    m = ConvNet().to(cuda)
    x = torch.randn(B, 1, 28, 28, device=cuda)
    yo = convnet_features(x, m.conv1, m.conv2, 0.0, True)
    assert yo.shape == (B, 9216) and yo.dtype == torch.float32
    g = torch.randn_like(yo)
    yr, ref = _ref_grads(x, m, g, _NAMES)
    torch.testing.assert_close(yo, yr.float().to(cuda), rtol=1e-5, atol=1e-5)
    ours = torch.autograd.grad(yo, [dict(m.named_parameters())[n] for n in _NAMES], g)
    for name, a, b in zip(_NAMES, ours, ref):
        rel = float((a - b).norm() / b.norm())
        assert rel < 1e-5, (name, rel)


def test_convnet_features_dropout(cuda):
    """Dropout2d inside the fused kernel: whole (n, c) planes dropped at rate p,
    kept planes scaled by 1/(1-p), the backward routes gradient only through
    kept planes (checked against the fp64 composition with the same mask)."""
    from distributed_compute_pytorch_amd.models import ConvNet
    from distributed_compute_pytorch_amd.ops import convnet_features

    torch.manual_seed(1)
    m = ConvNet().to(cuda)
    x = torch.randn(64, 1, 28, 28, device=cuda)
    yo = convnet_features(x, m.conv1, m.conv2, 0.25, True)
    base = _features_ref(x, m)[0].float().to(cuda).view(64, 64, 144)
    planes = yo.detach().view(64, 64, 144)
    nz = base.abs().sum(2) > 0
    kept = planes.abs().sum(2) > 0
    frac = (kept & nz).sum().item() / nz.sum().item()
    assert 0.65 < frac < 0.85, frac
    scale = kept.float() * (4.0 / 3.0)
    torch.testing.assert_close(planes, base * scale[:, :, None], rtol=1e-5, atol=1e-5)
    g = torch.randn_like(yo)
    names = ["conv1.weight", "conv2.weight", "conv2.bias"]
    ours = torch.autograd.grad(yo, [dict(m.named_parameters())[n] for n in names], g)
    _, ref = _ref_grads(x, m, g, names, scale)
    for n, a, b in zip(names, ours, ref):
        assert float((a - b).norm() / b.norm()) < 1e-5, n


@pytest.mark.parametrize("M,K,N", [(128, 9216, 128), (128, 128, 10), (37, 300, 20), (256, 9216, 128), (5, 16, 3)])
def test_fc32_matches_fp64(cuda, M, K, N):
    """The head's fp32-MFMA Linear (csrc/kernels/fc32.hip): forward (K-split +
    reduce for fc1's K = 9216), data gradient, weight gradient and bias
    gradient vs an fp64 reference; exact fp32 products (no xf32), so only
    summation order differs."""
    from distributed_compute_pytorch_amd.ops.convnet import fc32

    g = torch.Generator().manual_seed(M + K + N)
    lin = torch.nn.Linear(K, N).to(cuda)
    x = torch.randn(M, K, generator=g).to(cuda).requires_grad_(True)
    gy = torch.randn(M, N, generator=g).to(cuda)
    y = fc32(x, lin)
    y.backward(gy)
    xd, wd, bd = x.detach().double(), lin.weight.detach().double(), lin.bias.detach().double()
    yr = xd @ wd.t() + bd
    torch.testing.assert_close(y.double(), yr, rtol=2e-5, atol=2e-5 * K ** 0.5)
    torch.testing.assert_close(x.grad.double(), gy.double() @ wd, rtol=2e-5, atol=2e-5 * N ** 0.5)
    torch.testing.assert_close(lin.weight.grad.double(), gy.double().t() @ xd, rtol=2e-5, atol=2e-5 * M ** 0.5)
    torch.testing.assert_close(lin.bias.grad.double(), gy.double().sum(0), rtol=2e-5, atol=2e-5 * M ** 0.5)
    # deterministic: the K-split partials are summed in a fixed order
    assert torch.equal(fc32(x.detach(), lin), y.detach())
