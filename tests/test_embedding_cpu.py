"""FusedEmbedding (ops/embedding.py): forward and weight gradient equal
torch.nn.Embedding's (the scatter backward is the HIP-graph-safe replacement
for ATen's sort + host-sized segment pass)."""
import torch
from torch import nn

from distributed_compute_pytorch_amd.ops.embedding import FusedEmbedding


def test_fused_embedding_matches_torch():
    torch.manual_seed(0)
    ref = nn.Embedding(97, 24)
    ours = FusedEmbedding(97, 24)
    ours.load_state_dict(ref.state_dict())
    idx = torch.randint(0, 97, (5, 33))
    idx[0, :5] = 3  # repeated ids accumulate
    g = torch.randn(5, 33, 24)
    ref(idx).backward(g)
    y = ours(idx)
    y.backward(g)
    torch.testing.assert_close(y, ref(idx))
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-5)
    assert list(ours.state_dict()) == ["weight"]


def test_fused_embedding_tied_head_accumulates():
    torch.manual_seed(1)
    ours = FusedEmbedding(50, 8)
    ref = nn.Embedding(50, 8)
    ref.load_state_dict(ours.state_dict())
    idx = torch.randint(0, 50, (4, 7))
    for m in (ours, ref):
        x = m(idx)
        logits = torch.nn.functional.linear(x, m.weight)
        logits.square().mean().backward()
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-6)


def test_fused_embedding_deterministic_mode_uses_sorted_backward():
    torch.manual_seed(2)
    ours = FusedEmbedding(30, 6)
    idx = torch.randint(0, 30, (3, 9))
    prev = torch.are_deterministic_algorithms_enabled()
    try:
        torch.use_deterministic_algorithms(True)
        y = ours(idx)
        # F.embedding's own autograd node, not the atomic scatter
        assert "EmbeddingBackward" in type(y.grad_fn).__name__
    finally:
        torch.use_deterministic_algorithms(prev)
    assert "EmbeddingBackward" not in type(ours(idx).grad_fn).__name__


def test_fused_embedding_inplace_accumulation_sees_complete_grad():
    """Second backward onto an existing .grad: the scatter adds in place and
    returns None; the AccumulateGrad post-hook (what the DDP Reducer hangs on)
    still fires once, after every contribution of the tied weight is in."""
    import torch.nn.functional as F

    torch.manual_seed(2)
    ours = FusedEmbedding(40, 8)
    ref = nn.Embedding(40, 8)
    ref.load_state_dict(ours.state_dict())
    seen = []
    node = torch.autograd.graph.get_gradient_edge(ours.weight).node
    node.register_hook(lambda gi, go: seen.append(ours.weight.grad.clone()))
    for k in range(3):
        idx = torch.randint(0, 40, (4, 9))
        for m in (ours, ref):
            F.linear(m(idx), m.weight).square().mean().backward()
        assert len(seen) == k + 1
        torch.testing.assert_close(seen[-1], ref.weight.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-6)
    # a tensor hook on the parameter must see every contribution: no in-place shortcut then
    h = ours.weight.register_hook(lambda g: g)
    ours.weight.grad = None
    ref.weight.grad = None
    for _ in range(2):
        idx = torch.randint(0, 40, (4, 9))
        for m in (ours, ref):
            F.linear(m(idx), m.weight).square().mean().backward()
    h.remove()
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-6)


def test_autograd_grad_leaves_populated_grad_untouched():
    """a backward that does not accumulate into the
    parameter (autograd.grad w.r.t. the input only, backward(inputs=...)
    without it, autograd.grad w.r.t. the parameter) must neither add into an
    already populated .grad nor return None for the parameter."""
    torch.manual_seed(3)
    emb = FusedEmbedding(40, 6)
    idx = torch.randint(0, 40, (3, 5))
    emb.weight.grad = torch.ones_like(emb.weight)  # e.g. zero_grad(set_to_none=False) + mid-accumulation
    before = emb.weight.grad.clone()
    x = emb(idx)
    h = x * torch.linspace(0.5, 1.5, 6)
    # gradient w.r.t. the embedding OUTPUT only (input-saliency style)
    (gx,) = torch.autograd.grad(h.square().sum(), x, retain_graph=True)
    assert gx.shape == x.shape
    torch.testing.assert_close(emb.weight.grad, before)
    # gradient w.r.t. the parameter: returned, .grad untouched
    (gw,) = torch.autograd.grad(h.square().sum(), emb.weight, retain_graph=True)
    ref = nn.Embedding(40, 6)
    ref.load_state_dict(emb.state_dict())
    (gref,) = torch.autograd.grad((ref(idx) * torch.linspace(0.5, 1.5, 6)).square().sum(), ref.weight)
    torch.testing.assert_close(gw, gref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(emb.weight.grad, before)
    # a real backward still accumulates (in place) into the populated .grad
    h.square().sum().backward()
    torch.testing.assert_close(emb.weight.grad, before + gref, rtol=1e-5, atol=1e-5)
