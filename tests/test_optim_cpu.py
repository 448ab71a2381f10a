"""CPU path of the fused optimizers vs torch.optim (same math as the HIP kernels)."""
import pytest
import torch

import distributed_compute_pytorch_amd as dcp

SHAPES = [(7, 3), (100,), (2, 3, 4, 5), (1,)]


def _run(cls_ours, cls_ref, kw, dtype=torch.float32, steps=4):
    g = torch.Generator().manual_seed(0)
    base = [torch.randn(s, generator=g) for s in SHAPES]
    p1 = [b.clone().requires_grad_() for b in base]
    p2 = [b.clone().to(dtype).requires_grad_() for b in base]
    o1, o2 = cls_ref(p1, **kw), cls_ours(p2, **kw)
    for _ in range(steps):
        grads = [torch.randn(s, generator=g) for s in SHAPES]
        for a, b, gr in zip(p1, p2, grads):
            a.grad = gr.clone()
            b.grad = gr.to(dtype)
        o1.step()
        o2.step()
    return p1, p2, o1, o2


@pytest.mark.parametrize("kw", [dict(lr=0.1), dict(lr=0.1, momentum=0.9), dict(lr=0.1, momentum=0.9, nesterov=True),
                                dict(lr=0.1, momentum=0.9, weight_decay=1e-2, dampening=0.1),
                                dict(lr=0.1, momentum=0.5, maximize=True)])
def test_sgd(kw):
    p1, p2, o1, o2 = _run(dcp.optim.SGD, torch.optim.SGD, kw)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    if kw.get("momentum"):
        torch.testing.assert_close(o2.state[p2[0]]["momentum_buffer"], o1.state[p1[0]]["momentum_buffer"])


@pytest.mark.parametrize("name,kw", [("Adam", {}), ("Adam", {"weight_decay": 0.1}), ("AdamW", {}),
                                     ("Adam", {"amsgrad": True}), ("AdamW", {"maximize": True}),
                                     ("Adadelta", {}), ("Adadelta", {"lr": 1e-3, "weight_decay": 0.01})])
def test_adaptive(name, kw):
    p1, p2, o1, o2 = _run(getattr(dcp.optim, name), getattr(torch.optim, name), kw)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    sd1, sd2 = o1.state_dict(), o2.state_dict()
    for k in sd1["state"]:
        assert set(sd1["state"][k]) == set(sd2["state"][k])
        for kk in sd1["state"][k]:
            torch.testing.assert_close(sd2["state"][k][kk].float(), sd1["state"][k][kk].float(), rtol=1e-5,
                                       atol=1e-6)


def test_state_dict_roundtrip_into_torch():
    p1, p2, o1, o2 = _run(dcp.optim.Adam, torch.optim.Adam, {})
    o3 = torch.optim.Adam([q.detach().clone().requires_grad_() for q in p2])
    o3.load_state_dict(o2.state_dict())  # torch accepts our layout


def test_bf16_params():
    p1, p2, _, _ = _run(dcp.optim.SGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9), dtype=torch.bfloat16)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(b.float(), a, rtol=3e-2, atol=3e-2)


def test_clip_grad_norm_cpu():
    ps = [torch.nn.Parameter(torch.randn(s)) for s in SHAPES]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for p, q in zip(ps, qs):
        p.grad = torch.randn_like(p) * 3
        q.grad = p.grad.clone()
    n1 = torch.nn.utils.clip_grad_norm_(ps, 1.0)
    n2 = dcp.optim.clip_grad_norm_(qs, 1.0)
    torch.testing.assert_close(n2.float(), n1, rtol=1e-5, atol=1e-6)
    for p, q in zip(ps, qs):
        torch.testing.assert_close(q.grad, p.grad, rtol=1e-5, atol=1e-6)


def test_mt_copy_cpu():
    from distributed_compute_pytorch_amd._ext import C

    src = [torch.randn(5, 3), torch.randn(8, 4, 3, 3).contiguous(memory_format=torch.channels_last)]
    dst = [torch.empty_like(s) for s in src]
    C.mt_copy(src, dst, 2.0)
    for s, d in zip(src, dst):
        torch.testing.assert_close(d, s * 2)


def test_fused_adam_shadow_list_cpu():
    """fused_adam's optional bf16 shadow list holds the updated params (host path)."""
    from distributed_compute_pytorch_amd._ext import C

    torch.manual_seed(0)
    ps = [torch.randn(37), torch.randn(8, 16)]
    gs = [torch.randn_like(p) for p in ps]
    ms = [torch.zeros_like(p) for p in ps]
    vs = [torch.zeros_like(p) for p in ps]
    sh = [torch.empty_like(p, dtype=torch.bfloat16) for p in ps]
    ref = [p.clone().requires_grad_(True) for p in ps]
    C.fused_adam(ps, gs, ms, vs, [], 1e-2, 0.9, 0.999, 1e-8, 0.01, 1.0, False, True, False, 1.0, sh)
    opt = torch.optim.AdamW(ref, lr=1e-2, weight_decay=0.01)
    for r, g in zip(ref, gs):
        r.grad = g.clone()
    opt.step()
    for p, r, s in zip(ps, ref, sh):
        torch.testing.assert_close(p, r.detach(), rtol=1e-6, atol=1e-6)
        assert torch.equal(s, p.to(torch.bfloat16))


@pytest.mark.parametrize("name", ["Adam", "AdamW"])
def test_adam_mixed_chunked_and_full_steps(name):
    """Overlap-mode steps (one chunk per deferred bucket: ``_step(ids)``) mixed
    with whole-group steps (``_step(None)``) keep one step counter per
    parameter: the cached plans of both kinds cover the same parameters, and
    a plan whose counters the other took over is rebuilt, not reused stale."""
    g = torch.Generator().manual_seed(1)
    base = [torch.randn(s, generator=g) for s in SHAPES]
    p1 = [b.clone().requires_grad_() for b in base]
    p2 = [b.clone().requires_grad_() for b in base]
    o1, o2 = getattr(torch.optim, name)(p1, lr=0.01), getattr(dcp.optim, name)(p2, lr=0.01)
    ids_a = {id(p) for p in p2[:2]}
    ids_b = {id(p) for p in p2[2:]}
    pattern = [None, "chunks", "chunks", "chunks", None, "chunks", None, None]
    for b in p2:  # fixed gradient addresses, as DDP's bucket views are
        b.grad = torch.zeros_like(b)
    for kind in pattern:
        grads = [torch.randn(s, generator=g) for s in SHAPES]
        for a, b, gr in zip(p1, p2, grads):
            a.grad = gr.clone()
            b.grad.copy_(gr)
        o1.step()
        with torch.no_grad():
            if kind is None:
                o2._step(None, 1.0)
            else:
                o2._step(ids_a, 1.0)
                o2._step(ids_b, 1.0)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
        assert float(o2.state[b]["step"]) == float(o1.state[a]["step"]) == len(pattern)
