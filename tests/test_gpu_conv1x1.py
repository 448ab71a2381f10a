"""MFMA 1x1-convolution GEMMs (csrc/kernels/gemm.hip) vs plain PyTorch fp32
references of the same ops: forward (+BN-apply/ReLU prologue, +column-sum
epilogue), dgrad, wgrad, the fused BN→ReLU→conv autograd function, and a
ResNet bottleneck stage with the GEMM path on vs off."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # (N, H, W, Cin, Cout)
    (2, 8, 8, 64, 64),      # M = 128: one tile
    (3, 7, 7, 64, 256),     # M = 147: ragged last tile
    (4, 14, 14, 256, 64),
    (2, 9, 11, 128, 128),
    (8, 28, 28, 512, 128),  # several k-stages, persistent tiles
    (1, 5, 5, 192, 320),    # N not a multiple of 128 (BN = 64 tiles)
]


def _x(n, h, w, c, dev, gen):
    return torch.randn(n, c, h, w, generator=gen, device="cpu").to(dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.fixture(params=[0, 2], ids=["ring", "deep"])
def nt_deep(request):
    """gemm_tune nt_deep: 2 = the 3-slot 256 x 128 ring on every plain / stats
    1x1 forward (N % 128 == 0)."""
    from distributed_compute_pytorch_amd._ext import C as _C

    old = _C.gemm_tune_get("nt_deep")
    _C.gemm_tune("nt_deep", request.param)
    yield request.param
    _C.gemm_tune("nt_deep", old)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv1x1_fwd_stats(cuda, shape, nt_deep):
    from distributed_compute_pytorch_amd._ext import C as _C

    n, h, w, ci, co = shape
    g = torch.Generator().manual_seed(1)
    x = _x(n, h, w, ci, cuda, g)
    wt = (torch.randn(co, ci, generator=g) / ci ** 0.5).to(cuda).to(torch.bfloat16)
    y, st = _C.conv1x1_fwd(x, wt, None, None, False, True)
    ref = F.conv2d(x.float(), wt.float()[:, :, None, None])
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 1e-2
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(st[:co], yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(st[co:], (yf * yf).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("shape", SHAPES[:4])
def test_conv1x1_prologue(cuda, shape):
    from distributed_compute_pytorch_amd._ext import C as _C

    n, h, w, ci, co = shape
    g = torch.Generator().manual_seed(2)
    x = _x(n, h, w, ci, cuda, g)
    wt = (torch.randn(co, ci, generator=g) / ci ** 0.5).to(cuda).to(torch.bfloat16)
    sc = (torch.rand(ci, generator=g) + 0.5).to(cuda)
    sf = torch.randn(ci, generator=g).to(cuda)
    y, _ = _C.conv1x1_fwd(x, wt, sc, sf, True, False)
    a = torch.relu(x.float() * sc[None, :, None, None] + sf[None, :, None, None]).to(torch.bfloat16)
    ref = F.conv2d(a.float(), wt.float()[:, :, None, None])
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("shape", SHAPES)
def test_conv1x1_dgrad_wgrad(cuda, shape):
    from distributed_compute_pytorch_amd._ext import C as _C

    n, h, w, ci, co = shape
    g = torch.Generator().manual_seed(3)
    x = _x(n, h, w, ci, cuda, g)
    gy = _x(n, h, w, co, cuda, g)
    wt = (torch.randn(co, ci, generator=g) / ci ** 0.5).to(cuda).to(torch.bfloat16)
    dx = _C.conv1x1_dgrad(gy, wt.t().contiguous())
    ref_dx = F.conv_transpose2d(gy.float(), wt.float()[:, :, None, None])
    assert dx.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dx, ref_dx) < 1e-2
    dw = _C.conv1x1_wgrad(gy, x)
    ref_dw = torch.einsum("nchw,nkhw->ck", gy.float(), x.float())
    assert dw.dtype == torch.float32 and dw.shape == (co, ci)
    assert _rel(dw, ref_dw) < 1e-3
    # wgrad with the BN+ReLU prologue on x
    sc = (torch.rand(ci, generator=g) + 0.5).to(cuda)
    sf = torch.randn(ci, generator=g).to(cuda)
    dw2 = _C.conv1x1_wgrad(gy, x, sc, sf, True)
    a = torch.relu(x.float() * sc[None, :, None, None] + sf[None, :, None, None]).to(torch.bfloat16).float()
    assert _rel(dw2, torch.einsum("nchw,nkhw->ck", gy.float(), a)) < 1e-3


def test_bn_relu_conv1x1_autograd(cuda):
    """Fused BN(train)→ReLU→conv1x1 vs the fp32 ATen composition on the same
    bf16 input: output, every gradient, running statistics."""
    from torch import nn

    from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d
    from distributed_compute_pytorch_amd.ops.conv import bn_relu_conv1x1

    g = torch.Generator().manual_seed(4)
    n, h, w, ci, co = 8, 14, 14, 128, 256
    x = (_x(n, h, w, ci, cuda, g).float() * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn = BatchNormAct2d(ci, act=True, fused=True).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv = nn.Conv2d(ci, co, 1, bias=False).to(cuda)
    ref_bn = nn.BatchNorm2d(ci).to(cuda)
    ref_bn.load_state_dict(bn.state_dict())
    ref_conv = nn.Conv2d(ci, co, 1, bias=False).to(cuda)
    ref_conv.load_state_dict(conv.state_dict())

    xa = x.detach().clone().requires_grad_(True)
    z, st = bn_relu_conv1x1(xa, bn, conv.weight, stats=True)
    gz = _x(n, h, w, co, cuda, g)
    z.backward(gz)

    xr = x.detach().float().clone().requires_grad_(True)
    zr = ref_conv(torch.relu(ref_bn(xr)).to(torch.bfloat16).float())
    zr.backward(gz.float())

    assert _rel(z, zr) < 1.5e-2
    zf = z.float().permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(st[:co], zf.sum(0), rtol=1e-4, atol=1e-1)
    assert _rel(xa.grad, xr.grad) < 3e-2
    assert _rel(bn.weight.grad, ref_bn.weight.grad) < 3e-2
    assert _rel(bn.bias.grad, ref_bn.bias.grad) < 3e-2
    assert conv.weight.grad.dtype == torch.float32
    assert _rel(conv.weight.grad, ref_conv.weight.grad) < 2e-2
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-3, atol=1e-3)
    assert int(bn.num_batches_tracked) == 1


def test_resnet_stage_gemm_path_matches(cuda):
    """bf16 autocast training step of a small bottleneck ResNet with the GEMM
    path on vs off (same fused BN kernels otherwise), both measured against an
    fp32 run of the same weights: the GEMM path must be no less accurate than
    the MIOpen path (bf16 rounding compounds through the network, so the two
    bf16 runs are compared through their error to fp32, not to each other)."""
    from distributed_compute_pytorch_amd.models import resnet18_like

    torch.manual_seed(0)
    a = resnet18_like(num_classes=10, fused_bn=True, fused_gemm=True).to(cuda).to(memory_format=torch.channels_last)
    b = resnet18_like(num_classes=10, fused_bn=True, fused_gemm=False).to(cuda).to(memory_format=torch.channels_last)
    r = resnet18_like(num_classes=10, fused_bn=False).to(cuda).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    r.load_state_dict(a.state_dict())
    g = torch.Generator().manual_seed(0)
    x = torch.randn(16, 3, 64, 64, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), generator=g).to(cuda)
    losses = []
    for m, amp in ((a, True), (b, True), (r, False)):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        losses.append(float(loss))
    assert abs(losses[0] - losses[2]) < 3 * abs(losses[1] - losses[2]) + 2e-2
    for (n, p), q, s_ in zip(a.named_parameters(), b.parameters(), r.parameters()):
        assert p.grad is not None and p.grad.dtype == torch.float32, n
        ea, eb = _rel(p.grad, s_.grad), _rel(q.grad, s_.grad)
        assert ea < 1.5 * eb + 0.03, (n, ea, eb)
    for (n, x1), x2 in zip(a.named_buffers(), r.buffers()):
        torch.testing.assert_close(x1.float(), x2.float(), rtol=3e-2, atol=3e-2, msg=n)


@pytest.mark.parametrize("shape", [  # (N, H, W, Cin, Cout, k, stride, pad)
    (2, 8, 8, 64, 64, 3, 1, 1), (3, 7, 9, 128, 64, 3, 1, 1), (4, 14, 14, 64, 128, 3, 2, 1),
    (2, 15, 15, 128, 128, 3, 2, 1), (2, 6, 6, 64, 192, 1, 1, 0), (8, 28, 28, 128, 128, 3, 1, 1),
    # Cin = 64 kxk: the multi-tap kernel (two taps per 128-wide tile, last tile half past the taps)
    (4, 56, 56, 64, 64, 3, 1, 1), (3, 9, 11, 64, 64, 3, 1, 1), (2, 10, 10, 64, 64, 5, 1, 2),
    (2, 12, 12, 64, 192, 3, 2, 1)])
def test_conv_wgrad_gathered(cuda, shape):
    """Implicit-GEMM kxk weight gradient vs the fp32 ATen convolution backward."""
    from distributed_compute_pytorch_amd._ext import C as _C

    n, h, w, ci, co, k, s, p = shape
    g = torch.Generator().manual_seed(5)
    x = _x(n, h, w, ci, cuda, g)
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    gy = _x(n, ho, wo, co, cuda, g)
    dw = _C.conv_wgrad(gy, x, k, k, s, p)
    wt = torch.zeros(co, ci, k, k, device=cuda)
    ref = torch.ops.aten.convolution_backward(gy.float(), x.float(), wt, None, [s, s], [p, p], [1, 1], False, [0, 0],
                                              1, [False, True, False])[1]
    assert dw.shape == ref.shape and dw.dtype == torch.float32
    assert dw.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dw, ref) < 1e-3


def test_conv_kxk_autograd(cuda):
    from torch import nn

    from distributed_compute_pytorch_amd.ops.conv import conv_kxk

    g = torch.Generator().manual_seed(6)
    conv = nn.Conv2d(64, 128, 3, 2, 1, bias=False).to(cuda).to(memory_format=torch.channels_last)
    x = _x(4, 14, 14, 64, cuda, g).requires_grad_(True)
    y = conv_kxk(x, conv.weight, 2, 1)
    gy = _x(4, 7, 7, 128, cuda, g)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, conv.weight.detach().to(torch.bfloat16).float(), None, 2, 1)
    yr.backward(gy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(x.detach().float(), wr, None, 2, 1).backward(gy.float())
    assert conv.weight.grad.dtype == torch.float32 and _rel(conv.weight.grad, wr.grad) < 1e-3


@pytest.mark.parametrize("cin,cout,hw,k,stride,pad", [(64, 128, 14, 3, 1, 1), (64, 64, 9, 3, 2, 1), (128, 64, 7, 3, 1, 1),
                                                     (64, 128, 11, 1, 2, 0), (192, 64, 5, 3, 1, 1),
                                                     (128, 256, 10, 1, 2, 0), (128, 128, 14, 3, 2, 1),
                                                     (256, 64, 7, 3, 2, 1)])
def test_conv_kxk_gemm(cuda, cin, cout, hw, k, stride, pad):
    """Implicit-GEMM MFMA kxk conv (gemm.hip GATHER): forward + epilogue sums,
    data gradient (stride 1: the forward kernel on flipped weights; 3x3
    stride 2: the four parity classes in one launch, conv_dgrad_s2_multi),
    weight gradient, vs fp32 PyTorch on the same bf16 operands; ragged M."""
    from torch import nn

    from distributed_compute_pytorch_amd.ops.conv import conv_kxk_gemm

    g = torch.Generator().manual_seed(11)
    conv = nn.Conv2d(cin, cout, k, stride, pad, bias=False).to(cuda).to(memory_format=torch.channels_last)
    x = _x(3, hw, hw, cin, cuda, g).requires_grad_(True)
    y, st = conv_kxk_gemm(x, conv.weight, stride, pad, stats=True)
    ho = (hw + 2 * pad - k) // stride + 1
    assert y.shape == (3, cout, ho, ho) and y.is_contiguous(memory_format=torch.channels_last)
    gy = _x(3, ho, ho, cout, cuda, g)
    y.backward(gy)
    wb = conv.weight.detach().to(torch.bfloat16).float()
    xr = x.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wb, None, stride, pad)
    yr.backward(gy.float())
    assert _rel(y, yr) < 1e-2
    yf = y.float()
    ref_st = torch.cat([yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))])
    assert _rel(st, ref_st) < 1e-4
    assert _rel(x.grad, xr.grad) < 1e-2
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(x.detach().float(), wr, None, stride, pad).backward(gy.float())
    assert conv.weight.grad.dtype == torch.float32 and _rel(conv.weight.grad, wr.grad) < 1e-3


@pytest.mark.parametrize("k,stride,pad,sums,co", [(3, 1, 1, True, 128), (3, 2, 1, False, 128), (1, 1, 0, True, 128),
                                                  (3, 1, 1, True, 64)])
def test_bn_relu_conv_fused_autograd(cuda, k, stride, pad, sums, co):
    """BN(train)→ReLU→conv as one node (BN backward reduced in the dgrad GEMM's
    epilogue) vs the fp32 ATen composition on the same bf16 input. co = 64:
    the direct 3x3 / 64-channel kernels, the dgrad's RED epilogue included."""
    from torch import nn

    from distributed_compute_pytorch_amd.ops.batchnorm import BatchNormAct2d
    from distributed_compute_pytorch_amd.ops.conv import bn_relu_conv

    g = torch.Generator().manual_seed(13)
    n, h, w, ci = 4, 12, 12, 64
    x = (_x(n, h, w, ci, cuda, g).float() * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn = BatchNormAct2d(ci, act=True, fused=True).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv = nn.Conv2d(ci, co, k, stride, pad, bias=False).to(cuda).to(memory_format=torch.channels_last)
    ref_bn = nn.BatchNorm2d(ci).to(cuda)
    ref_bn.load_state_dict(bn.state_dict())
    ref_conv = nn.Conv2d(ci, co, k, stride, pad, bias=False).to(cuda)
    ref_conv.load_state_dict(conv.state_dict())

    xa = x.detach().clone().requires_grad_(True)
    s_in = None
    if sums:
        xf = x.float()
        s_in = torch.cat([xf.sum((0, 2, 3)), (xf * xf).sum((0, 2, 3))]).contiguous()
    z, st = bn_relu_conv(xa, bn, conv.weight, k, stride, pad, sums=s_in, stats=True)
    gz = _x(n, z.shape[2], z.shape[3], co, cuda, g)
    z.backward(gz)

    xr = x.detach().float().clone().requires_grad_(True)
    zr = ref_conv(torch.relu(ref_bn(xr)).to(torch.bfloat16).float())
    zr.backward(gz.float())

    assert _rel(z, zr) < 1.5e-2
    zf = z.float()
    assert _rel(st, torch.cat([zf.sum((0, 2, 3)), (zf * zf).sum((0, 2, 3))])) < 1e-3
    assert _rel(xa.grad, xr.grad) < 3e-2
    assert _rel(bn.weight.grad, ref_bn.weight.grad) < 3e-2
    assert _rel(bn.bias.grad, ref_bn.bias.grad) < 3e-2
    assert conv.weight.grad.dtype == torch.float32 and _rel(conv.weight.grad, ref_conv.weight.grad) < 2e-2
    torch.testing.assert_close(bn.running_mean, ref_bn.running_mean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_var, ref_bn.running_var, rtol=1e-3, atol=1e-3)


def test_conv_weight_bf16_layouts(cuda):
    from distributed_compute_pytorch_amd._ext import C as _C

    g = torch.Generator().manual_seed(14)
    w = torch.randn(96, 64, 3, 3, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    wf, wd = _C.conv_weight_bf16(w)
    wb = w.to(torch.bfloat16)
    assert torch.equal(wf, wb.permute(0, 2, 3, 1).contiguous())
    assert torch.equal(wd, wb.flip(2, 3).permute(1, 2, 3, 0).contiguous())


@pytest.mark.parametrize("n,h,w", [(2, 56, 56), (3, 7, 9), (2, 5, 62), (4, 13, 2), (5, 30, 31), (2, 17, 40)])
def test_conv3x3_c64_direct(cuda, n, h, w):
    """Direct 3x3 / 64-channel kernels (halo in LDS): forward + BN sums, the
    stride-1 data gradient (same kernel on flipped weights) and the weight
    gradient (conv3x3_c64_wgrad_kernel) vs
    fp32 PyTorch on the same bf16 operands, rectangular and ragged row tiles."""
    from torch import nn

    from distributed_compute_pytorch_amd.ops.conv import conv_kxk_gemm

    g = torch.Generator().manual_seed(21)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).to(cuda).to(memory_format=torch.channels_last)
    x = _x(n, h, w, 64, cuda, g).requires_grad_(True)
    y, st = conv_kxk_gemm(x, conv.weight, 1, 1, stats=True)
    gy = _x(n, h, w, 64, cuda, g)
    y.backward(gy)
    wb = conv.weight.detach().to(torch.bfloat16).float()
    xr = x.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wb, None, 1, 1)
    yr.backward(gy.float())
    assert _rel(y, yr) < 1e-2
    yf = y.float()
    ref_st = torch.cat([yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))])
    assert _rel(st, ref_st) < 1e-4
    assert _rel(x.grad, xr.grad) < 1e-2
    # weight gradient: the direct halo kernel (conv3x3_c64_wgrad_kernel) + slab reduction
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(x.detach().float(), wr, None, 1, 1).backward(gy.float())
    assert conv.weight.grad.dtype == torch.float32 and _rel(conv.weight.grad, wr.grad) < 1e-3


@pytest.fixture
def pro_pipe():
    """gemm_tune pro_pipe = 1: the BN-prologue GEMMs on the BK = 64 pipelined
    stage loop (256-row tiles) instead of the BK = 32 ring."""
    from distributed_compute_pytorch_amd._ext import C as _C

    old = _C.gemm_tune_get("pro_pipe")
    _C.gemm_tune("pro_pipe", 1)
    yield
    _C.gemm_tune("pro_pipe", old)


@pytest.mark.parametrize("shape", SHAPES + [(16, 14, 14, 256, 1024), (4, 7, 7, 512, 2048)])
@pytest.mark.parametrize("relu", [True, False])
def test_conv1x1_prologue_pipelined(cuda, shape, relu, pro_pipe):
    """BN(+ReLU) prologue on the pipelined BK = 64 loop: output and the
    Σy / Σy² epilogue against an fp32 reference of the same bf16 operand."""
    from distributed_compute_pytorch_amd._ext import C as _C

    n, h, w, ci, co = shape
    g = torch.Generator().manual_seed(12)
    x = _x(n, h, w, ci, cuda, g)
    wt = (torch.randn(co, ci, generator=g) / ci ** 0.5).to(cuda).to(torch.bfloat16)
    sc = (torch.rand(ci, generator=g) + 0.5).to(cuda)
    sf = torch.randn(ci, generator=g).to(cuda)
    y, st = _C.conv1x1_fwd(x, wt, sc, sf, relu, True)
    a = x.float() * sc[None, :, None, None] + sf[None, :, None, None]
    a = (torch.relu(a) if relu else a).to(torch.bfloat16)
    ref = F.conv2d(a.float(), wt.float()[:, :, None, None])
    assert _rel(y, ref) < 1e-2
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, co)
    torch.testing.assert_close(st[:co], yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(st[co:], (yf * yf).sum(0), rtol=1e-4, atol=1e-2)
    # bit-identical to the BK = 32 ring's prologue (same fp32 expression, same bf16 operand)
    _C.gemm_tune("pro_pipe", 0)
    y0, _ = _C.conv1x1_fwd(x, wt, sc, sf, relu, False)
    _C.gemm_tune("pro_pipe", 1)
    assert _rel(y, y0) < 1e-2
