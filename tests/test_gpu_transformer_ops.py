"""Fused LayerNorm and vocab cross-entropy kernels vs fp32 PyTorch references."""
import contextlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 128, 768), (33, 1024), (7, 4096), (5, 3, 8), (1000, 512), (16, 1024, 768), (3001, 256), (5, 3, 768), (1037, 768)])
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


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 7, 4096, 1000003])
def test_dropout_statistics_and_backward(cuda, dtype, n):
    from distributed_compute_pytorch_amd.ops import dropout_add, fused_dropout

    torch.manual_seed(0)
    x = torch.randn(n, device=cuda, dtype=dtype).requires_grad_()
    y = fused_dropout(x, 0.3)
    kept = (y != 0)
    if n > 1000:
        assert abs(kept.float().mean().item() - 0.7) < 0.02
    torch.testing.assert_close(y[kept].float(), (x[kept] / 0.7).float(), rtol=1e-2, atol=1e-2)
    y.backward(torch.ones_like(y))
    # gradient mask == forward mask (regenerated from the same counter)
    assert torch.equal(x.grad != 0, kept)
    r = torch.randn(n, device=cuda, dtype=dtype)
    torch.manual_seed(5)
    z = dropout_add(x.detach(), r, 0.3)
    torch.manual_seed(5)
    z2 = fused_dropout(x.detach(), 0.3) + r
    torch.testing.assert_close(z.float(), z2.float(), rtol=1e-2, atol=1e-2)


def test_feature_dropout(cuda):
    from distributed_compute_pytorch_amd.ops import fused_feature_dropout

    x = torch.randn(64, 32, 6, 6, device=cuda, requires_grad=True)
    y = fused_feature_dropout(x, 0.25)
    per_ch = (y.detach() != 0).reshape(64, 32, -1)
    assert torch.all(per_ch.all(-1) | (~per_ch).all(-1))  # whole channels kept or dropped
    frac = per_ch.all(-1).float().mean().item()
    assert abs(frac - 0.75) < 0.06
    y.sum().backward()
    torch.testing.assert_close((x.grad != 0), (y.detach() != 0))


def test_layer_norm_autocast_fp32_in_bf16_out(cuda):
    from distributed_compute_pytorch_amd.ops import FusedLayerNorm

    torch.manual_seed(0)
    m = FusedLayerNorm(768).to(cuda)
    ref = torch.nn.LayerNorm(768).to(cuda)
    x = torch.randn(4, 64, 768, device=cuda, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
        yr = ref(xr)
    assert y.dtype == torch.bfloat16 and x.dtype == torch.float32
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype))
    yr.backward(g)
    assert x.grad.dtype == torch.float32
    torch.testing.assert_close(x.grad, xr.grad, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layer_norm_dual_output_sums_both_gradients(cuda, dtype):
    """fused_layer_norm_dual(alias_output=True): (ln(x), alias of ln(x)); both
    outputs' gradients are summed as the LN backward loads dy — vs fp64
    PyTorch of ln(x)·a + ln(x)·c."""
    from distributed_compute_pytorch_amd.ops.layernorm import fused_layer_norm_dual

    torch.manual_seed(1)
    D = 768
    w = (1 + 0.1 * torch.randn(D, device=cuda)).requires_grad_()
    b = (0.1 * torch.randn(D, device=cuda)).requires_grad_()
    x = torch.randn(6, 50, D, device=cuda).to(dtype).requires_grad_()
    a, c = torch.randn(6, 50, D, device=cuda), torch.randn(6, 50, D, device=cuda)
    y, alias = fused_layer_norm_dual(x, (D,), w, b, alias_output=True)
    assert alias.data_ptr() == y.data_ptr()
    ((y.float() * a).sum() + (alias.float() * c).sum()).backward()
    xr = x.detach().double().requires_grad_()
    wr, br = w.detach().double().requires_grad_(), b.detach().double().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br)
    ((yr * a.double()).sum() + (yr * c.double()).sum()).backward()
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=6e-2)
    torch.testing.assert_close(x.grad.double(), xr.grad, **tol)
    ptol = dict(rtol=1e-3, atol=1e-2) if dtype == torch.float32 else dict(rtol=2e-2, atol=0.3)
    torch.testing.assert_close(w.grad.double(), wr.grad, **ptol)
    torch.testing.assert_close(b.grad.double(), br.grad, **ptol)


def test_bert_dual_ln_matches_plain_ln(cuda):
    """The fused BERT layers with dual-output post-LNs compute the same
    gradients as the same layers with plain LNs (fp32, tight)."""
    from distributed_compute_pytorch_amd.models import bert as bm

    torch.manual_seed(0)
    cfg = bm.BertConfig(vocab_size=128, hidden=256, layers=2, heads=4, intermediate=512, max_position=64,
                        dropout=0.0, fused=True)
    m = bm.BertForPreTraining(cfg).to(cuda)
    ids = torch.randint(0, 128, (2, 64), device=cuda)
    labels = torch.randint(0, 128, (2, 64), device=cuda)
    m(ids, mlm_labels=labels).backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    orig = bm.FusedLayerNorm.forward_dual_out
    # plain LN: the two consumers share one autograd output (autograd adds their gradients)
    bm.FusedLayerNorm.forward_dual_out = lambda self, x: (lambda y: (y, y))(self(x))
    try:
        m(ids, mlm_labels=labels).backward()
    finally:
        bm.FusedLayerNorm.forward_dual_out = orig
    for n, p in m.named_parameters():
        if p.grad is not None:
            torch.testing.assert_close(p.grad, grads[n], rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.parametrize("model", ["gpt2", "bert"])
def test_dropout_add_ln_fusion_matches_unfused(cuda, model, monkeypatch):
    """Residual dropout + LayerNorm as one kernel each way (LnDropAdd) vs the
    separate dropout_add + LN kernels, with dropout on: the fused op draws the
    same Philox masks (same seed draw per dropout), so loss and every gradient
    agree (bf16 autocast, same rounding points)."""
    from distributed_compute_pytorch_amd.models import bert as bm
    from distributed_compute_pytorch_amd.models import gpt2 as g2
    from distributed_compute_pytorch_amd.ops import layernorm as lnm

    torch.manual_seed(0)
    if model == "gpt2":
        m = g2.GPT2(g2.GPT2Config(vocab_size=512, n_positions=128, n_embd=256, n_layer=2, n_head=4, dropout=0.2)).to(cuda)
        ids = torch.randint(0, 512, (2, 128), device=cuda)
        run = lambda: m(ids, ids)  # noqa: E731
    else:
        m = bm.BertForPreTraining(bm.BertConfig(vocab_size=128, hidden=256, layers=2, heads=4, intermediate=512,
                                                max_position=128, dropout=0.2)).to(cuda)
        ids = torch.randint(0, 128, (2, 128), device=cuda)
        labels = torch.randint(0, 128, (2, 128), device=cuda)
        run = lambda: m(ids, mlm_labels=labels)  # noqa: E731
    m.train()
    out = {}
    for fuse in (False, True):
        monkeypatch.setattr(lnm, "FUSE_DADD_LN", fuse)
        m.zero_grad(set_to_none=True)
        torch.manual_seed(7)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = run()
        loss.backward()
        out[fuse] = (loss.detach().float(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
    torch.testing.assert_close(out[True][0], out[False][0], rtol=1e-3, atol=1e-3)
    # (the key bias's gradient is zero in exact arithmetic — softmax ignores a
    # per-query constant — so it is rounding noise: compared against the scale
    # of the other gradients instead)
    mx = max(float(g.norm()) for g in out[False][1].values())
    for n, g in out[False][1].items():
        d = float((out[True][1][n] - g).norm())
        if float(g.norm()) < 1e-3 * mx:
            assert d < 1e-3 * mx, (n, d, mx)
        else:
            assert d / float(g.norm()) < 2e-2, (n, d / float(g.norm()))


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("rdtype", [torch.float32, torch.bfloat16])
def test_dropout_add_layer_norm_op(cuda, mode, rdtype):
    """dropout_add_layer_norm vs dropout_add then the (dual) LayerNorm under
    the same seed: outputs and the gradients of branch, residual, gamma, beta."""
    from distributed_compute_pytorch_amd.ops.dropout import dropout_add
    from distributed_compute_pytorch_amd.ops.layernorm import FusedLayerNorm, dropout_add_layer_norm

    torch.manual_seed(3)
    D = 768
    ln = FusedLayerNorm(D).to(cuda)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    br = torch.randn(4, 37, D, device=cuda).to(torch.bfloat16)
    res = torch.randn(4, 37, D, device=cuda).to(rdtype)
    gy = torch.randn(4, 37, D, device=cuda)
    g2 = torch.randn(4, 37, D, device=cuda)
    outs = []
    for fused in (True, False):
        b_ = br.clone().requires_grad_()
        r_ = res.clone().requires_grad_()
        ln.zero_grad(set_to_none=True)
        torch.manual_seed(11)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                o = dropout_add_layer_norm(b_, r_, ln, 0.3, True, mode)
            else:
                x = dropout_add(b_, r_, 0.3, True)
                o = ln(x) if mode == 0 else (ln.forward_dual(x) if mode == 1 else ln.forward_dual_out(x))
        if mode == 0:
            (o.float() * gy).sum().backward()
            ys = [o]
        else:
            ((o[0].float() * gy).sum() + (o[1].float() * g2).sum()).backward()
            ys = list(o)
        outs.append(([y.detach().float() for y in ys], b_.grad.float(), r_.grad.float(), ln.weight.grad.clone(),
                     ln.bias.grad.clone()))
    (yf, bf, rf, wf, bbf), (yu, bu, ru, wu, bbu) = outs
    for a, b in zip(yf, yu):
        torch.testing.assert_close(a, b, rtol=0, atol=0)  # same kernels' math, same masks: identical
    for a, b in ((bf, bu), (rf, ru), (wf, wu), (bbf, bbu)):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layer_norm_dual_sums_both_gradients(cuda, dtype):
    """fused_layer_norm_dual: (ln(x), alias of x); the alias's gradient is added
    into dx inside the LN backward kernel — vs fp64 PyTorch of ln(x)·a + x·b."""
    from distributed_compute_pytorch_amd.ops.layernorm import fused_layer_norm_dual

    torch.manual_seed(0)
    D = 768
    w = (1 + 0.1 * torch.randn(D, device=cuda)).requires_grad_()
    b = (0.1 * torch.randn(D, device=cuda)).requires_grad_()
    x = torch.randn(6, 50, D, device=cuda).to(dtype).requires_grad_()
    a, c = torch.randn(6, 50, D, device=cuda), torch.randn(6, 50, D, device=cuda)
    y, alias = fused_layer_norm_dual(x, (D,), w, b)
    assert alias.data_ptr() == x.data_ptr()
    ((y.float() * a).sum() + (alias.float() * c).sum()).backward()
    xr = x.detach().double().requires_grad_()
    wr, br = w.detach().double().requires_grad_(), b.detach().double().requires_grad_()
    ((torch.nn.functional.layer_norm(xr, (D,), wr, br) * a.double()).sum() + (xr * c.double()).sum()).backward()
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(x.grad.double(), xr.grad, **tol)
    # bf16: y (hence dy) is bf16-rounded, dγ / dβ sum 300 such rows
    ptol = dict(rtol=1e-3, atol=1e-2) if dtype == torch.float32 else dict(rtol=2e-2, atol=0.15)
    torch.testing.assert_close(w.grad.double(), wr.grad, **ptol)
    torch.testing.assert_close(b.grad.double(), br.grad, **ptol)


def test_gpt2_dual_ln_matches_plain_ln(cuda):
    """The fused GPT-2 block with dual-output LNs computes the same gradients
    as the same block with plain LNs (same kernels, one add moved into the LN
    backward): fp32, tight tolerance."""
    from distributed_compute_pytorch_amd.models import gpt2 as g2

    torch.manual_seed(0)
    cfg = g2.GPT2Config(vocab_size=512, n_positions=64, n_embd=256, n_layer=2, n_head=4, dropout=0.0, fused=True)
    m = g2.GPT2(cfg).to(cuda)
    idx = torch.randint(0, 512, (2, 64), device=cuda)
    m(idx, idx).backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    orig = g2.Block.forward

    def plain(self, x):
        x = self._dadd(self.attn(self.ln_1(x)), x, self.p, self.training)
        return self._dadd(self.mlp(self.ln_2(x)), x, self.p, self.training)

    g2.Block.forward = plain
    fuse = g2.ln_mod.FUSE_DADD_LN
    g2.ln_mod.FUSE_DADD_LN = False  # the per-block loop (Block.forward), not forward_pending
    try:
        m(idx, idx).backward()
    finally:
        g2.Block.forward = orig
        g2.ln_mod.FUSE_DADD_LN = fuse
    for n, p in m.named_parameters():
        if p.grad is not None:
            torch.testing.assert_close(p.grad, grads[n], rtol=1e-5, atol=1e-6, msg=n)


def test_dropout_add_mixed_dtypes(cuda):
    from distributed_compute_pytorch_amd.ops import dropout_add

    x = torch.randn(1 << 16, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(1 << 16, device=cuda, dtype=torch.float32, requires_grad=True)
    y = dropout_add(x, r, 0.2)
    assert y.dtype == torch.float32
    y.backward(torch.ones_like(y))
    assert x.grad.dtype == torch.bfloat16 and r.grad.dtype == torch.float32
    kept = (y.detach() - r.detach()) != 0
    assert torch.equal(x.grad != 0, kept)
    torch.testing.assert_close(r.grad, torch.ones_like(r))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("log_probs", [True, False])
def test_eval_metrics(cuda, dtype, log_probs):
    from distributed_compute_pytorch_amd.ops import EvalMetrics

    torch.manual_seed(0)
    m = EvalMetrics(cuda, log_probs=log_probs)
    tot_loss, tot_corr, tot_n = 0.0, 0, 0
    for _ in range(3):
        s = torch.randn(777, 1000, device=cuda)
        if log_probs:
            s = torch.log_softmax(s, 1)
        y = torch.randint(0, 1000, (777,), device=cuda)
        y[:5] = -100
        s = s.to(dtype)
        m.update(s, y)
        sf = s.float()
        lp = sf if log_probs else torch.log_softmax(sf, 1)
        tot_loss += F.nll_loss(lp, y, ignore_index=-100, reduction="sum").item()
        tot_corr += (sf.argmax(1).eq(y) & y.ne(-100)).sum().item()
        tot_n += y.ne(-100).sum().item()
    avg, acc, n = m.compute(all_reduce=False)
    assert n == tot_n
    assert abs(avg - tot_loss / tot_n) < 1e-3 * max(1, abs(avg))
    assert abs(acc - tot_corr / tot_n) < 1e-9


@pytest.mark.parametrize("shape", [(4096, 768), (1000, 3072), (7, 64)])
def test_colsum_matches_torch(cuda, shape):
    from distributed_compute_pytorch_amd._ext import C as _C

    g = torch.Generator().manual_seed(11)
    x = torch.randn(*shape, generator=g).to(cuda).to(torch.bfloat16)
    out = _C.colsum(x)
    ref = x.float().sum(0)
    assert out.dtype == torch.float32
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("ours", ["pp", "ring"])
def test_fused_linear_matches_fp32(cuda, monkeypatch, ours):
    from torch import nn

    from distributed_compute_pytorch_amd.ops import linear as lin_mod
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear

    # our GEMM (ping-pong or ring) is what must be validated: no per-shape
    # autotune to hipBLASLt
    monkeypatch.setattr(lin_mod, "_AUTOTUNE", False)
    monkeypatch.setattr(lin_mod, "_CHOICE", {})
    monkeypatch.setattr(lin_mod, "_DEFAULT_OURS", ours)

    torch.manual_seed(0)
    lin = FusedLinear(256, 384).to(cuda)
    ref = nn.Linear(256, 384).to(cuda)
    ref.load_state_dict(lin.state_dict())
    g = torch.Generator().manual_seed(12)
    x = torch.randn(4, 64, 256, generator=g).to(cuda)
    gy = torch.randn(4, 64, 384, generator=g).to(cuda).to(torch.bfloat16)
    xa = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lin(xa)
    y.backward(gy)
    xr = x.to(torch.bfloat16).float().requires_grad_(True)
    yr = F.linear(xr, ref.weight.to(torch.bfloat16).float(), ref.bias.to(torch.bfloat16).float())
    yr.backward(gy.float())
    wr = ref.weight.detach().clone().requires_grad_(True)
    br = ref.bias.detach().clone().requires_grad_(True)
    F.linear(x.to(torch.bfloat16).float(), wr, br).backward(gy.float())

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm())

    assert y.dtype == torch.bfloat16 and rel(y, yr) < 1e-2
    assert rel(xa.grad, xr.grad) < 1e-2
    assert lin.weight.grad.dtype == torch.float32 and rel(lin.weight.grad, wr.grad) < 1e-2
    assert lin.bias.grad.dtype == torch.float32 and rel(lin.bias.grad, br.grad) < 1e-3


@pytest.mark.parametrize("ours", ["pp", "ring"])
@pytest.mark.parametrize("approximate", ["none", "tanh"])
@pytest.mark.parametrize("rows,fin,fout", [(4 * 64, 256, 1024), (37, 128, 520), (8192, 768, 3072)])
def test_fused_linear_gelu_matches_fp32(cuda, approximate, rows, fin, fout, monkeypatch, ours):
    """FusedLinear.forward_gelu (GEMM + gelu.hip forward; GELU backward with the
    bias column sums fused) vs an fp32 PyTorch reference on the same bf16 inputs."""
    from torch import nn

    from distributed_compute_pytorch_amd.ops import linear as lin_mod
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear

    monkeypatch.setattr(lin_mod, "_AUTOTUNE", False)
    monkeypatch.setattr(lin_mod, "_CHOICE", {})
    monkeypatch.setattr(lin_mod, "_DEFAULT_OURS", ours)

    torch.manual_seed(0)
    lin = FusedLinear(fin, fout).to(cuda)
    ref = nn.Linear(fin, fout).to(cuda)
    ref.load_state_dict(lin.state_dict())
    g = torch.Generator().manual_seed(7)
    x = torch.randn(rows, fin, generator=g).to(cuda)
    gy = torch.randn(rows, fout, generator=g).to(cuda).to(torch.bfloat16)
    xa = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lin.forward_gelu(xa, approximate)
    y.backward(gy)
    xr = x.to(torch.bfloat16).float().requires_grad_(True)
    wr = ref.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = ref.bias.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.gelu(F.linear(xr, wr, br), approximate=approximate)
    yr.backward(gy.float())

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm())

    assert y.dtype == torch.bfloat16 and rel(y, yr) < 1e-2
    assert rel(xa.grad, xr.grad) < 1e-2
    assert lin.weight.grad.dtype == torch.float32 and rel(lin.weight.grad, wr.grad) < 1e-2
    assert lin.bias.grad.dtype == torch.float32 and rel(lin.bias.grad, br.grad) < 1e-2


def test_gelu_kernels_elementwise(cuda):
    """Raw gelu_fwd / gelu_bwd vs fp32 ATen on a wide value range (no bias grad)."""
    from distributed_compute_pytorch_amd._ext import C

    h = (torch.linspace(-12, 12, 64 * 1000, device=cuda)).to(torch.bfloat16).view(1000, 64)
    gy = torch.randn(1000, 64, device=cuda).to(torch.bfloat16)
    for approx in ("none", "tanh"):
        y = C.gelu_fwd(h, approx == "tanh")
        torch.testing.assert_close(y.float(), F.gelu(h.float(), approximate=approx), rtol=1e-2, atol=1e-2)
        hr = h.float().requires_grad_(True)
        F.gelu(hr, approximate=approx).backward(gy.float())
        gh, db = C.gelu_bwd(gy, h, approx == "tanh", False)
        assert db is None
        torch.testing.assert_close(gh.float(), hr.grad, rtol=1e-2, atol=2e-2)
        gh2, db2 = C.gelu_bwd(gy, h, approx == "tanh", True)
        torch.testing.assert_close(db2, gh2.float().sum(0), rtol=1e-4, atol=1e-3)


def test_fused_linear_in_place_accumulation_and_weight_cache(cuda):
    """Micro-steps under ``accumulate_grads_in_place`` (what DDP.no_sync enables)
    add dW / db inside the kernels: the accumulated .grad must equal autograd's
    own accumulation; the cached bf16 weight must follow optimizer updates."""
    import copy

    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear, accumulate_grads_in_place

    torch.manual_seed(0)
    a = FusedLinear(256, 384).to(cuda)
    b = copy.deepcopy(a)
    g = torch.Generator().manual_seed(13)
    xs = [torch.randn(2, 64, 256, generator=g).to(cuda) for _ in range(3)]
    gys = [torch.randn(2, 64, 384, generator=g).to(cuda).to(torch.bfloat16) for _ in range(3)]
    for fwd in ("forward", "forward_gelu"):  # plain Linear, Linear+GELU (bias grad in the GELU kernel)
        a.zero_grad(set_to_none=True)
        b.zero_grad(set_to_none=True)
        for k, (x, gy) in enumerate(zip(xs, gys)):
            for m, inplace in ((a, True), (b, False)):
                ctx = accumulate_grads_in_place() if (inplace and k < 2) else contextlib.nullcontext()
                with ctx, torch.autocast("cuda", dtype=torch.bfloat16):
                    y = getattr(m, fwd)(x)
                with ctx:
                    y.backward(gy)
        torch.testing.assert_close(a.weight.grad, b.weight.grad, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(a.bias.grad, b.bias.grad, rtol=1e-5, atol=1e-5)
    # weight cache: an optimizer step must invalidate the bf16 copy
    opt = dcp.optim.SGD(a.parameters(), lr=0.5)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y0 = a(xs[0])
    opt.step()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = a(xs[0])
    # the same GEMM on a freshly cast weight: bit-equal iff the cache followed the step
    from distributed_compute_pytorch_amd._ext import C as _C

    ref = _C.linear_fwd(xs[0].to(torch.bfloat16).contiguous(), a.weight.detach().to(torch.bfloat16),
                        a.bias.detach().float().contiguous(), 0)[0]
    assert not torch.equal(y0, y1)
    torch.testing.assert_close(y1, ref, rtol=0, atol=0)


@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16])
def test_layer_norm_in_place_accumulation(cuda, xdtype):
    """Under ``accumulate_grads_in_place`` the LayerNorm finalize kernel adds
    dγ / dβ into the existing fp32 .grad (no AccumulateGrad add): the result
    must equal autograd's own accumulation over the same micro-steps."""
    import copy

    from distributed_compute_pytorch_amd.ops.layernorm import FusedLayerNorm
    from distributed_compute_pytorch_amd.ops.linear import accumulate_grads_in_place

    torch.manual_seed(0)
    a = FusedLayerNorm(768).to(cuda)
    with torch.no_grad():
        a.weight.uniform_(0.5, 1.5)
        a.bias.uniform_(-0.5, 0.5)
    b = copy.deepcopy(a)
    g = torch.Generator().manual_seed(17)
    xs = [torch.randn(4, 100, 768, generator=g).to(cuda).to(xdtype) for _ in range(3)]
    gys = [torch.randn(4, 100, 768, generator=g).to(cuda).to(xdtype) for _ in range(3)]
    dxa, dxb = [], []
    for k, (x, gy) in enumerate(zip(xs, gys)):
        for m, inplace, dxs in ((a, True, dxa), (b, False, dxb)):
            xx = x.clone().requires_grad_(True)
            ctx = accumulate_grads_in_place() if (inplace and k < 2) else contextlib.nullcontext()
            with ctx:
                m(xx).backward(gy)
            dxs.append(xx.grad)
    for u, v in zip(dxa, dxb):
        torch.testing.assert_close(u, v, rtol=0, atol=0)
    torch.testing.assert_close(a.weight.grad, b.weight.grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(a.bias.grad, b.bias.grad, rtol=1e-5, atol=1e-4)
    # the sum of the three micro-steps against an fp32 PyTorch reference
    wr = b.weight.detach().clone().requires_grad_(True)
    br = b.bias.detach().clone().requires_grad_(True)
    for x, gy in zip(xs, gys):
        F.layer_norm(x.float(), (768,), wr, br, 1e-5).backward(gy.float())
    tol = 2e-2 if xdtype == torch.bfloat16 else 1e-3
    torch.testing.assert_close(a.weight.grad, wr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(a.bias.grad, br.grad, rtol=tol, atol=tol)


def test_adamw_writes_bf16_shadow_weights(cuda):
    """FusedLinear registers its bf16 weight copy; the fused AdamW step rewrites
    it in the update kernel (RNE, identical to a fresh .to(bf16)) and the next
    forward reuses it without a cast."""
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear
    from distributed_compute_pytorch_amd.optim.fused import fresh_bf16_shadow

    torch.manual_seed(0)
    a = FusedLinear(256, 384).to(cuda)
    opt = dcp.optim.AdamW(a.parameters(), lr=1e-2)
    x = torch.randn(4, 64, 256, device=cuda)
    for _ in range(3):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = a.forward_gelu(x, "tanh")
        y.float().square().mean().backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        sw = fresh_bf16_shadow(a.weight)
        assert sw is not None and fresh_bf16_shadow(a.bias) is not None
        torch.testing.assert_close(sw, a.weight.detach().to(torch.bfloat16), rtol=0, atol=0)
        torch.testing.assert_close(fresh_bf16_shadow(a.bias), a.bias.detach().to(torch.bfloat16), rtol=0, atol=0)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = a(x)
    assert a._w16_cache[1] is fresh_bf16_shadow(a.weight)
    # the forward GEMM reads the shadow: fp32 reference on the same bf16
    # operands (bias added in fp32 before the one bf16 rounding)
    ref = (x.to(torch.bfloat16).float() @ a.weight.to(torch.bfloat16).float().t() + a.bias.float())
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)
    with torch.no_grad():  # an out-of-band write invalidates the shadow
        a.weight.mul_(0.5)
    assert fresh_bf16_shadow(a.weight) is None


@pytest.mark.parametrize("lin_big", [0, 2])
@pytest.mark.parametrize("gelu", [0, 1, 2])
@pytest.mark.parametrize("rows,fin,fout", [(1000, 256, 192), (2048, 768, 2304), (333, 64, 128), (700, 128, 512)])
def test_linear_fwd_epilogues_match_fp32(cuda, gelu, rows, fin, fout, lin_big):
    """gemm_nt's Linear epilogues (bias before the bf16 rounding; + GELU tanh /
    erf from the rounded h) vs fp32 PyTorch on the same bf16 operands, on the
    128-row tiles and (lin_big=2, N % 256 == 0) the 256 x 256 tiles."""
    from distributed_compute_pytorch_amd._ext import C

    g = torch.Generator().manual_seed(3)
    x = torch.randn(rows, fin, generator=g).to(torch.bfloat16).to(cuda)
    w = (torch.randn(fout, fin, generator=g) / fin ** 0.5).to(torch.bfloat16).to(cuda)
    b = torch.randn(fout, generator=g).to(cuda)
    old = C.gemm_tune_get("lin_big")
    C.gemm_tune("lin_big", lin_big)
    try:
        out = C.linear_fwd(x, w, b, gelu)
    finally:
        C.gemm_tune("lin_big", old)
    h_ref = x.float() @ w.float().t() + b
    h = out[-1]
    assert h.dtype == torch.bfloat16 and h.shape == (rows, fout)
    torch.testing.assert_close(h.float(), h_ref, rtol=1e-2, atol=1e-2)
    if gelu:
        y_ref = F.gelu(h.float(), approximate="tanh" if gelu == 1 else "none")  # GELU of the stored h
        torch.testing.assert_close(out[0].float(), y_ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("pp", [False, True])
@pytest.mark.parametrize("tanh", [True, False])
@pytest.mark.parametrize("rows,n1,n2", [(1000, 512, 256), (4096, 3072, 768), (333, 128, 64), (700, 264, 128)])
def test_linear_dgrad_gelu_matches_fp32(cuda, tanh, rows, n1, n2, pp):
    """gemm.hip EPI 10/11 (ring) and gemm_pp.hip EPI 4/5 (ping-pong): gh =
    (gy·W2)·gelu'(h) and db = Σ gh, vs fp32 PyTorch on the same bf16 operands
    (gh of the bf16-rounded gy·W2)."""
    from distributed_compute_pytorch_amd._ext import C

    if not pp and n1 % 64:
        pytest.skip("the ring takes multiples of 64 columns")
    g = torch.Generator().manual_seed(5)
    gy = torch.randn(rows, n2, generator=g).to(torch.bfloat16).to(cuda)
    w2 = (torch.randn(n2, n1, generator=g) / n1 ** 0.5).to(torch.bfloat16).to(cuda)
    h = torch.randn(rows, n1, generator=g).to(torch.bfloat16).to(cuda)
    gh, db = C.linear_dgrad_gelu(gy, w2.t().contiguous(), h, tanh, pp=pp)
    dy = (gy.float() @ w2.float()).to(torch.bfloat16).float()
    hr = h.float().requires_grad_()
    torch.nn.functional.gelu(hr, approximate="tanh" if tanh else "none").backward(dy)
    torch.testing.assert_close(gh.float(), hr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(db, gh.float().sum(0), rtol=1e-4, atol=1e-3)
    acc = torch.ones(n1, device=cuda)
    C.linear_dgrad_gelu(gy, w2.t().contiguous(), h, tanh, accumulate_into=acc, pp=pp)
    torch.testing.assert_close(acc, 1 + gh.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("ours", ["pp", "ring", "blasfwd", "ppbwd"])
@pytest.mark.parametrize("approx", ["tanh", "none"])
def test_fused_mlp_matches_fp32(cuda, approx, monkeypatch, ours):
    """ops.linear.fused_mlp_gelu (one node: GELU forward in fc's epilogue,
    GELU backward + fc's bias sum in proj's dgrad epilogue) vs fp32 PyTorch of
    proj(gelu(fc(x))) on the same bf16-rounded parameters and input. The
    per-shape autotune is off so the fused node itself runs."""
    from distributed_compute_pytorch_amd.ops import linear as lin
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear, fused_mlp_gelu

    monkeypatch.setattr(lin, "_AUTOTUNE", False)
    monkeypatch.setattr(lin, "_CHOICE", {})
    monkeypatch.setattr(lin, "_DEFAULT_OURS", "ring" if ours in ("blasfwd", "ppbwd") else ours)
    if ours == "blasfwd":  # the fused node with fc's forward on hipBLASLt + the GELU kernel
        lin._CHOICE[("fwd_gelu", 1024, 256, 1024)] = "hipblaslt"
        lin._CHOICE[("mlp_bwd", 1024, 256, 1024)] = "ring"
    if ours == "ppbwd":  # the GELU backward in the ping-pong GEMM's epilogue
        lin._CHOICE[("mlp_bwd", 1024, 256, 1024)] = "pp"

    torch.manual_seed(0)
    fc, proj = FusedLinear(256, 1024).to(cuda), FusedLinear(1024, 256).to(cuda)
    with torch.no_grad():
        for p in (*fc.parameters(), *proj.parameters()):
            p.copy_(p.to(torch.bfloat16).float())
    x = torch.randn(8, 128, 256, device=cuda).to(torch.bfloat16).float().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = fused_mlp_gelu(x, fc, proj, approx)
    assert "MLPFn" in type(y.grad_fn).__name__
    g = torch.randn_like(y, dtype=torch.float32)
    y.float().backward(g)
    ref = [t.detach().clone().requires_grad_() for t in (x, fc.weight, fc.bias, proj.weight, proj.bias)]
    yr = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(ref[0], ref[1], ref[2]),
                                                             approximate=approx), ref[3], ref[4])
    yr.backward(g)
    assert (y.float() - yr).norm() / yr.norm() < 1e-2
    for got, want, name in ((x.grad, ref[0].grad, "x"), (fc.weight.grad, ref[1].grad, "w1"),
                            (fc.bias.grad, ref[2].grad, "b1"), (proj.weight.grad, ref[3].grad, "w2"),
                            (proj.bias.grad, ref[4].grad, "b2")):
        rel = float((got.float() - want).norm() / want.norm())
        assert rel < 2e-2, (name, rel)


def test_fused_linear_autograd_grad_leaves_populated_grad(cuda):
    """torch.autograd.grad(loss, x) with a populated .grad
    (set_to_none=False / mid-accumulation) must not add the weight gradient
    into .grad; autograd.grad w.r.t. the weight must return it."""
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear

    torch.manual_seed(0)
    lin = FusedLinear(256, 384).to(cuda)
    lin.weight.grad = torch.ones_like(lin.weight)
    lin.bias.grad = torch.ones_like(lin.bias)
    w0, b0 = lin.weight.grad.clone(), lin.bias.grad.clone()
    x = torch.randn(2, 64, 256, device=cuda, requires_grad=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = lin(x).float().square().mean()
    (gx,) = torch.autograd.grad(loss, x, retain_graph=True)
    assert gx.shape == x.shape and torch.isfinite(gx).all()
    assert torch.equal(lin.weight.grad, w0) and torch.equal(lin.bias.grad, b0)
    gw, gb = torch.autograd.grad(loss, [lin.weight, lin.bias], retain_graph=True)
    assert gw is not None and gb is not None and gw.abs().sum() > 0
    assert torch.equal(lin.weight.grad, w0) and torch.equal(lin.bias.grad, b0)
    loss.backward()
    torch.testing.assert_close(lin.weight.grad, w0 + gw, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(lin.bias.grad, b0 + gb, rtol=1e-4, atol=1e-5)
