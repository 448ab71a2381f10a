"""LinearWeightPrep (one-launch bf16 W / Wᵀ of Linear weights, packed groups,
padded vocabularies) and the fused LM head + cross-entropy node, against fp32
PyTorch references. Autotune off: our kernels are what runs (``_DEFAULT_OURS``
picks pp or the ring for the forward GEMMs; pp_xent = the head GEMM with the
cross-entropy partials in its epilogue where there is no bias, else the ring)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["pp", "ring", "pp_xent"])
def ours(request, monkeypatch):
    from distributed_compute_pytorch_amd.ops import linear

    monkeypatch.setattr(linear, "_AUTOTUNE", False)
    monkeypatch.setattr(linear, "_DEFAULT_OURS", request.param)
    monkeypatch.setattr(linear, "_CHOICE", {})
    return request.param


def _bf(t):
    return t.detach().to(torch.bfloat16)


def test_weight_prep_plan_linear_groups_and_padding(cuda):
    from distributed_compute_pytorch_amd._ext import C

    torch.manual_seed(0)
    ws = [torch.randn(r, c, device=cuda) for r, c in [(96, 64), (64, 128), (64, 128), (32, 128), (1003, 192)]]
    table, tiles, wb, wt = C.weight_prep_plan(ws, [1, 3, 1], [0, 0, 1024])
    C.weight_prep_run(table, tiles)
    torch.cuda.synchronize()
    assert len(wb) == len(wt) == 3
    exp = [ws[0], torch.cat(ws[1:4], 0), F.pad(ws[4], (0, 0, 0, 21))]
    for b, t, e in zip(wb, wt, exp):
        assert b.shape == e.shape and t.shape == e.t().shape
        assert torch.equal(b, _bf(e)) and torch.equal(t, _bf(e).t().contiguous())


def test_weight_prep_plan_rejects_bad_groups(cuda):
    from distributed_compute_pytorch_amd._ext import C

    ws = [torch.randn(64, 64, device=cuda), torch.randn(64, 128, device=cuda)]
    with pytest.raises(RuntimeError):
        C.weight_prep_plan(ws, [2])  # unequal input features in one group
    with pytest.raises(RuntimeError):
        C.weight_prep_plan(ws, [1])  # groups do not cover every weight
    with pytest.raises(RuntimeError):
        C.weight_prep_plan(ws, [1, 1], [32, 0])  # padding below the rows


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("M,K,V", [(256, 128, 1003), (1000, 192, 4097), (64, 64, 64)])
def test_lm_head_cross_entropy_matches_fp32(cuda, ours, bias, M, K, V):
    from distributed_compute_pytorch_amd.ops.linear import LinearWeightPrep
    from distributed_compute_pytorch_amd.ops.lm_head import lm_head_cross_entropy, padded_vocab

    torch.manual_seed(0)
    w = (torch.randn(V, K, device=cuda) * 0.05).requires_grad_()
    b = (torch.randn(V, device=cuda) * 0.1).requires_grad_() if bias else None
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16).requires_grad_()
    t = torch.randint(0, V, (M,), device=cuda)
    t[::7] = -100
    prep = LinearWeightPrep([(w,)], [padded_vocab(V)])
    prep.refresh()
    loss = lm_head_cross_entropy(x, w, b, t)
    loss.backward()
    # fp32 reference over the same bf16-rounded operands
    xr = x.detach().float().requires_grad_()
    wr = _bf(w).float().requires_grad_()
    br = b.detach().clone().requires_grad_() if bias else None
    lr = F.cross_entropy(F.linear(xr, wr, br), t, ignore_index=-100)
    lr.backward()
    torch.testing.assert_close(loss, lr, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * float(xr.grad.abs().max()))
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * float(wr.grad.abs().max()))
    if bias:
        torch.testing.assert_close(b.grad, br.grad, rtol=2e-2, atol=2e-2 * float(br.grad.abs().max()))


@pytest.mark.parametrize("wgrad", ["ring", "hipblaslt"])
def test_lm_head_accumulates_into_existing_grad(cuda, ours, wgrad):
    """A second backward adds its weight gradient into the fp32 .grad inside
    the GEMM (our wgrad's reduction pass, or hipBLASLt's beta = 1) — no
    separate add; rows past V are never written."""
    from distributed_compute_pytorch_amd.ops import linear
    from distributed_compute_pytorch_amd.ops.linear import LinearWeightPrep
    from distributed_compute_pytorch_amd.ops.lm_head import lm_head_cross_entropy

    torch.manual_seed(1)
    V, K, M = 1003, 128, 512
    linear._CHOICE[("head_wgrad", M, 1024, K)] = wgrad
    w = (torch.randn(V, K, device=cuda) * 0.05).requires_grad_()
    prep = LinearWeightPrep([(w,)], [1024])
    xs = [torch.randn(M, K, device=cuda, dtype=torch.bfloat16) for _ in range(2)]
    ts = [torch.randint(0, V, (M,), device=cuda) for _ in range(2)]
    gs = []
    for x, t in zip(xs, ts):
        prep.refresh()
        w.grad = None
        lm_head_cross_entropy(x, w, None, t).backward()
        gs.append(w.grad.clone())
    w.grad = None
    for x, t in zip(xs, ts):
        prep.refresh()
        lm_head_cross_entropy(x, w, None, t).backward()
    torch.testing.assert_close(w.grad, gs[0] + gs[1], rtol=1e-5, atol=1e-6)
    # and the first pass agrees with an fp32 reference of dW
    xr, wr = xs[0].float(), _bf(w).float().requires_grad_()
    F.cross_entropy(F.linear(xr, wr), ts[0]).backward()
    torch.testing.assert_close(gs[0], wr.grad, rtol=2e-2, atol=2e-2 * float(wr.grad.abs().max()))


def test_lm_head_second_backward_fails_loudly(cuda, ours):
    from distributed_compute_pytorch_amd.ops.linear import LinearWeightPrep
    from distributed_compute_pytorch_amd.ops.lm_head import lm_head_cross_entropy

    w = torch.randn(128, 64, device=cuda).requires_grad_()
    LinearWeightPrep([(w,)], [128]).refresh()
    x = torch.randn(64, 64, device=cuda, dtype=torch.bfloat16)
    loss = lm_head_cross_entropy(x, w, None, torch.randint(0, 128, (64,), device=cuda))
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError):
        loss.backward()  # the logits were overwritten by their gradient


def test_packed_linear_on_prep_matches_fp32(cuda, ours):
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear, LinearWeightPrep, packed_linear, prepped_linear

    torch.manual_seed(0)
    layers = [FusedLinear(256, 256).to(cuda) for _ in range(3)]
    prep = LinearWeightPrep([tuple(l.weight for l in layers)])
    prep.refresh()
    assert prepped_linear(tuple(l.weight for l in layers)) is not None
    x = torch.randn(4, 128, 256, device=cuda, dtype=torch.bfloat16).requires_grad_()
    y = packed_linear(x, layers)
    assert y.grad_fn is not None and "PackedLinear" in type(y.grad_fn).__name__
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    refs = [(_bf(l.weight).float().requires_grad_(), l.bias.detach().clone().requires_grad_()) for l in layers]
    yr = torch.cat([F.linear(xr, w, b) for w, b in refs], -1)
    yr.backward(g.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=5e-2)
    for l, (w, b) in zip(layers, refs):
        torch.testing.assert_close(l.weight.grad, w.grad, rtol=2e-2, atol=0.5)
        torch.testing.assert_close(l.bias.grad, b.grad, rtol=2e-2, atol=0.5)


def test_prep_views_go_stale_and_refresh(cuda):
    """Readers get the prepped views only while they hold the weights'
    current values: after an in-place update (autograd version) or a fused
    optimizer step (epoch), until the next refresh."""
    from distributed_compute_pytorch_amd import optim
    from distributed_compute_pytorch_amd.ops.linear import FusedLinear, LinearWeightPrep, prepped_linear

    lin = FusedLinear(128, 64).to(cuda)
    prep = LinearWeightPrep([(lin.weight,)])
    prep.refresh()
    wb, wt = prepped_linear((lin.weight,))
    assert torch.equal(wb, _bf(lin.weight))
    with torch.no_grad():
        lin.weight.mul_(2)
    assert prepped_linear((lin.weight,)) is None
    prep.refresh()
    wb, wt = prepped_linear((lin.weight,))
    assert torch.equal(wt, _bf(lin.weight).t().contiguous())
    opt = optim.AdamW(lin.parameters(), lr=0.1)
    lin.weight.grad = torch.randn_like(lin.weight)
    lin.bias.grad = torch.randn_like(lin.bias)
    opt.step()
    assert prepped_linear((lin.weight,)) is None
    prep.refresh()
    wb, _ = prepped_linear((lin.weight,))
    assert torch.equal(wb, _bf(lin.weight))


@pytest.mark.parametrize("name", ["gpt2", "bert"])
def test_model_step_uses_prep_and_head(cuda, name):
    """The fused models route their Linears, packed QKV and the LM head
    through the prep (no per-call weight cast / transpose)."""
    from distributed_compute_pytorch_amd import models
    from distributed_compute_pytorch_amd.ops import linear

    torch.manual_seed(0)
    if name == "gpt2":
        m = models.gpt2_small(n_layer=2).to(cuda)
        idx = torch.randint(0, 50257, (2, 128), device=cuda)
        args, kw = (idx, idx.roll(-1, 1)), {}
    else:
        m = models.bert_base(layers=2).to(cuda)
        ids = torch.randint(0, 30522, (2, 128), device=cuda)
        args = (ids,)
        kw = dict(mlm_positions=torch.randint(0, 128, (2, 20), device=cuda),
                  mlm_labels=torch.randint(0, 30522, (2, 20), device=cuda))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = m(*args, **kw)
    assert "LMHeadXent" in type(loss.grad_fn).__name__ or any(
        "LMHeadXent" in type(f[0]).__name__ for f in loss.grad_fn.next_functions if f[0] is not None)
    prep = m.__dict__["_linear_prep"]
    n_lin = sum(isinstance(x, linear.FusedLinear) for x in m.modules())
    members = sum(len(g) for g in prep.groups)
    assert members == n_lin + 1, (members, n_lin)  # every FusedLinear (packed ones as groups) + the head
    loss.backward()
    assert all(p.grad is not None for n, p in m.named_parameters() if "pooler" not in n and "nsp" not in n)


@pytest.mark.parametrize("M,K,N,V", [(512, 128, 1024, 1003), (1000, 192, 4160, 4097), (300, 64, 64, 64),
                                     (8192, 768, 50304, 50257)])
def test_lm_head_xent_fwd_partials_match_fp64(cuda, M, K, N, V):
    """The head GEMM's softmax-partials epilogue + merge: logits equal the plain
    ping-pong GEMM's bit for bit; lse and the per-row loss match an fp64
    log-sum-exp over the stored bf16 logits' first V columns (ignored targets
    give 0)."""
    from distributed_compute_pytorch_amd._ext import C

    torch.manual_seed(3)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.1).to(torch.bfloat16)
    w[V:] = 0  # the padded vocabulary rows, as LinearWeightPrep leaves them
    t = torch.randint(0, V, (M,), device=cuda)
    t[::5] = -100
    logits, loss, lse = C.lm_head_xent_fwd(x, w, t, -100, V)
    old = {k: C.gemm_tune_get(k) for k in ("pp_tile", "pp_sk")}
    try:  # the same one-tile 256 x 256 kernel without the partials (no 128 x 192 tiles, no split-K)
        C.gemm_tune("pp_tile", 1)
        C.gemm_tune("pp_sk", 0)
        ref_logits = C.gemm_pp(x, w, None, 0)[0]
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            C.gemm_tune(k, v)
    assert torch.equal(logits, ref_logits)
    lg = logits[:, :V].double()
    ref_lse = torch.logsumexp(lg, 1)
    keep = t != -100
    ref_loss = torch.where(keep, ref_lse - lg.gather(1, t.clamp_min(0)[:, None])[:, 0], torch.zeros_like(ref_lse))
    torch.testing.assert_close(lse.double(), ref_lse, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss.double(), ref_loss, rtol=1e-5, atol=1e-5)
