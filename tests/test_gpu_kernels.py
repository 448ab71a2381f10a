"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lists(dev, dtype, shapes, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [torch.randn(s, generator=g).to(dev, dtype) for s in shapes]


SHAPES = [(64, 3, 7, 7), (1000,), (2048, 1000), (5,), (3, 17), (1,), (8193,)]


@pytest.mark.parametrize("sd,dd", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                   (torch.bfloat16, torch.float32), (torch.float16, torch.float32)])
def test_mt_copy(cuda, sd, dd):
    from distributed_compute_pytorch_amd._ext import C

    src = _lists(cuda, sd, SHAPES)
    dst = [torch.empty_like(s, dtype=dd) for s in src]
    C.mt_copy(src, dst, 0.5)
    for s, d in zip(src, dst):
        torch.testing.assert_close(d.float(), (s.float() * 0.5).to(dd).float(), rtol=1e-2, atol=1e-2)


def test_mt_copy_channels_last(cuda):
    from distributed_compute_pytorch_amd._ext import C

    src = [torch.randn(8, 16, 5, 5, device=cuda).contiguous(memory_format=torch.channels_last)]
    dst = [torch.empty_like(src[0])]
    C.mt_copy(src, dst, 1.0)
    torch.testing.assert_close(dst[0], src[0])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nesterov,wd,mom", [(False, 0.0, 0.9), (True, 1e-4, 0.9), (False, 1e-4, 0.0)])
def test_fused_sgd_matches_torch(cuda, dtype, nesterov, wd, mom):
    import distributed_compute_pytorch_amd as dcp

    ref = [p.clone().float().requires_grad_() for p in _lists(cuda, dtype, SHAPES, 1)]
    ours = [p.detach().clone().to(dtype).requires_grad_() for p in ref]
    o1 = torch.optim.SGD(ref, lr=0.1, momentum=mom, weight_decay=wd, nesterov=nesterov)
    o2 = dcp.optim.SGD(ours, lr=0.1, momentum=mom, weight_decay=wd, nesterov=nesterov)
    for it in range(3):
        gs = _lists(cuda, torch.float32, SHAPES, 10 + it)
        for p, q, g in zip(ref, ours, gs):
            p.grad = g.clone()
            q.grad = g.to(dtype)
        o1.step()
        o2.step()
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    for p, q in zip(ref, ours):
        torch.testing.assert_close(q.detach().float(), p.detach(), rtol=tol, atol=tol)


@pytest.mark.parametrize("cls,kw", [("Adam", {}), ("AdamW", {"weight_decay": 0.01}), ("Adam", {"amsgrad": True}),
                                    ("Adadelta", {"lr": 1.0}), ("Adadelta", {"lr": 1e-3, "weight_decay": 0.1})])
def test_fused_adaptive_matches_torch(cuda, cls, kw):
    import distributed_compute_pytorch_amd as dcp

    ref = [p.clone().requires_grad_() for p in _lists(cuda, torch.float32, SHAPES, 2)]
    ours = [p.detach().clone().requires_grad_() for p in ref]
    o1 = getattr(torch.optim, cls)(ref, **kw)
    o2 = getattr(dcp.optim, cls)(ours, **kw)
    for it in range(4):
        gs = _lists(cuda, torch.float32, SHAPES, 20 + it)
        for p, q, g in zip(ref, ours, gs):
            p.grad = g.clone()
            q.grad = g.clone()
        o1.step()
        o2.step()
    for p, q in zip(ref, ours):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-5, atol=1e-6)
    # torch-compatible state layout
    s1, s2 = o1.state_dict(), o2.state_dict()
    assert s1["state"].keys() == s2["state"].keys()
    for k in s1["state"]:
        assert set(s1["state"][k].keys()) == set(s2["state"][k].keys())


def test_clip_grad_norm(cuda):
    import distributed_compute_pytorch_amd as dcp

    ps = [torch.nn.Parameter(t) for t in _lists(cuda, torch.float32, SHAPES, 3)]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for p, q, g in zip(ps, qs, _lists(cuda, torch.float32, SHAPES, 4)):
        p.grad = g.clone()
        q.grad = g.clone()
    n1 = torch.nn.utils.clip_grad_norm_(ps, 1.0)
    n2 = dcp.optim.clip_grad_norm_(qs, 1.0)
    torch.testing.assert_close(n2, n1, rtol=1e-4, atol=1e-5)
    for p, q in zip(ps, qs):
        torch.testing.assert_close(q.grad, p.grad, rtol=1e-4, atol=1e-6)
