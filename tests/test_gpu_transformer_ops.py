"""Fused LayerNorm and vocab cross-entropy kernels vs fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 128, 768), (33, 1024), (7, 4096), (5, 3, 8), (1000, 512)])
@pytest.mark.parametrize("affine", [True, False])
def test_layer_norm(cuda, dtype, shape, affine):
    from distributed_compute_pytorch_amd.ops import fused_layer_norm

    torch.manual_seed(0)
    D = shape[-1]
    x = (torch.randn(shape, device=cuda) * 3 + 1).to(dtype)
    w = (torch.rand(D, device=cuda) + 0.5).requires_grad_() if affine else None
    b = torch.randn(D, device=cuda).requires_grad_() if affine else None
    gy = torch.randn(shape, device=cuda).to(dtype)
    xr = x.float().requires_grad_()
    wr = w.detach().clone().requires_grad_() if affine else None
    br = b.detach().clone().requires_grad_() if affine else None
    yr = F.layer_norm(xr, (D,), wr, br, 1e-5)
    yr.backward(gy.float())
    xo = x.detach().clone().requires_grad_()
    yo = fused_layer_norm(xo, (D,), w, b, 1e-5)
    yo.backward(gy)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(yo.float(), yr, **tol)
    torch.testing.assert_close(xo.grad.float(), xr.grad, **tol)
    if affine:
        rows = x.numel() // D
        atol = 1e-3 * rows ** 0.5 if dtype == torch.float32 else 0.05 * rows ** 0.5
        torch.testing.assert_close(w.grad, wr.grad, rtol=1e-3, atol=atol)
        torch.testing.assert_close(b.grad, br.grad, rtol=1e-3, atol=atol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,V", [(64, 50257), (37, 30522), (16, 7), (5, 1000), (3, 65536)])
@pytest.mark.parametrize("reduction,ls", [("mean", 0.0), ("sum", 0.0), ("none", 0.0), ("mean", 0.1)])
def test_cross_entropy(cuda, dtype, rows, V, reduction, ls):
    from distributed_compute_pytorch_amd.ops import fused_cross_entropy

    torch.manual_seed(0)
    logits = (torch.randn(rows, V, device=cuda) * 4).to(dtype)
    target = torch.randint(0, V, (rows,), device=cuda)
    target[0] = -100  # ignored
    lr = logits.float().requires_grad_()
    ref = F.cross_entropy(lr, target, ignore_index=-100, reduction=reduction, label_smoothing=ls)
    go = torch.randn_like(ref)
    ref.backward(go)
    lo = logits.detach().clone().requires_grad_()
    out = fused_cross_entropy(lo, target, -100, reduction, ls)
    out.backward(go)
    torch.testing.assert_close(out.float(), ref, rtol=1e-4, atol=1e-4)
    tol = dict(rtol=1e-4, atol=1e-6) if dtype == torch.float32 else dict(rtol=2e-2, atol=1e-3)
    torch.testing.assert_close(lo.grad.float(), lr.grad, **tol)


def test_cross_entropy_unaligned_rows(cuda):
    """Odd row stride (V=50257, bf16): row starts are not 16-B aligned."""
    from distributed_compute_pytorch_amd.ops import fused_cross_entropy

    logits = torch.randn(9, 50257, device=cuda, dtype=torch.bfloat16)
    target = torch.randint(0, 50257, (9,), device=cuda)
    sl = logits[1:]  # storage offset 50257 elements: misaligned start
    torch.testing.assert_close(fused_cross_entropy(sl, target[1:]), F.cross_entropy(sl.float(), target[1:]),
                               rtol=1e-4, atol=1e-4)
