"""MFMA flash attention (csrc/kernels/attention.hip) vs a plain PyTorch fp32
reference of the same op (softmax(QKᵀ/8 [+causal]) → dropout → ·V), forward
and all three gradients; dropout uses the kernels' own keep-mask rebuilt by
``dropout_keep_mask`` (integer torch ops)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # B, H, T, causal, p
    (2, 3, 128, False, 0.0),
    (2, 3, 128, True, 0.0),
    (1, 2, 192, False, 0.1),   # T not a multiple of the 128-query block
    (2, 2, 256, True, 0.1),
    (1, 4, 512, False, 0.1),
    (1, 2, 192, True, 0.1),    # causal, last key tile half outside T
    (1, 2, 256, False, 0.6),   # keep threshold >= 128 (the other SWAR compare)
    (1, 2, 128, True, 0.5),    # threshold exactly 128
]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _reference(q, k, v, H, causal, p, keep):
    B, T, C = q.shape

    def heads(t):
        return t.float().view(B, T, H, 64).transpose(1, 2)

    s = heads(q) @ heads(k).transpose(-1, -2) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    P = torch.softmax(s, -1)
    if p > 0:
        from distributed_compute_pytorch_amd.ops.attention import dropout_p_effective

        P = P * keep / (1 - dropout_p_effective(p))
    return (P @ heads(v)).transpose(1, 2).reshape(B, T, C)


@pytest.mark.parametrize("case", CASES)
def test_flash_attn_matches_reference(cuda, case):
    from distributed_compute_pytorch_amd.ops.attention import dropout_keep_mask, flash_attn

    B, H, T, causal, p = case
    C = H * 64
    g = torch.Generator().manual_seed(7)
    q, k, v, do = (torch.randn(B, T, C, generator=g).to(cuda).to(torch.bfloat16) for _ in range(4))
    seed = 1234567891234
    keep = dropout_keep_mask(B, H, T, p, seed, cuda).float() if p > 0 else None
    if p > 0:  # the hash keeps ≈ 1-p of the elements
        assert abs(float(keep.mean()) - (1 - p)) < 0.01
    qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = flash_attn(qa, ka, va, H, causal, p, seed)
    o.backward(do)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ref = _reference(qr, kr, vr, H, causal, p, keep)
    ref.backward(do.float())
    assert o.shape == (B, T, C) and o.dtype == torch.bfloat16
    assert _rel(o, ref) < 1e-2, _rel(o, ref)
    for name, a, r in (("dq", qa.grad, qr.grad), ("dk", ka.grad, kr.grad), ("dv", va.grad, vr.grad)):
        assert _rel(a, r) < 2e-2, (name, _rel(a, r))


def test_flash_attn_qkv_packed(cuda):
    from distributed_compute_pytorch_amd.ops.attention import flash_attn, flash_attn_qkv

    B, H, T = 2, 4, 256
    C = H * 64
    g = torch.Generator().manual_seed(8)
    qkv = torch.randn(B, T, 3 * C, generator=g).to(cuda).to(torch.bfloat16)
    do = torch.randn(B, T, C, generator=g).to(cuda).to(torch.bfloat16)
    a = qkv.clone().requires_grad_(True)
    o = flash_attn_qkv(a, H, True, 0.1, 42)
    o.backward(do)
    parts = [qkv[..., i * C:(i + 1) * C].contiguous().requires_grad_(True) for i in range(3)]
    o2 = flash_attn(*parts, H, True, 0.1, 42)
    o2.backward(do)
    assert torch.equal(o, o2)
    assert torch.equal(a.grad, torch.cat([t.grad for t in parts], dim=2))


@pytest.mark.parametrize("case", [(2, 3, 256, False, 0.1), (1, 2, 192, True, 0.3), (1, 2, 128, False, 0.7)])
def test_stored_keep_bits_match_oracle(cuda, case):
    """The forward's stored keep bits (read by both backward kernels) decode
    to exactly the hash oracle's mask (causal: on and below the diagonal)."""
    from distributed_compute_pytorch_amd.ops.attention import dropout_keep_mask, flash_attn_keep_bits

    B, H, T, causal, p = case
    C = H * 64
    g = torch.Generator().manual_seed(9)
    q, k, v = (torch.randn(B, T, C, generator=g).to(cuda).to(torch.bfloat16) for _ in range(3))
    seed = 987654321
    got = flash_attn_keep_bits(q, k, v, H, causal, p, seed)
    want = dropout_keep_mask(B, H, T, p, seed, cuda)
    if causal:
        want = want & torch.ones(T, T, dtype=torch.bool, device=cuda).tril()
    assert torch.equal(got, want), int((got != want).sum())



def test_no_grad_forward_skips_keep_bits(cuda):
    """Without a backward to follow (no_grad) the forward stores no keep bits;
    its output is the same as with them."""
    from distributed_compute_pytorch_amd._ext import C as _C
    from distributed_compute_pytorch_amd.ops.attention import flash_attn

    B, H, T = 2, 2, 256
    C = H * 64
    g = torch.Generator().manual_seed(10)
    q, k, v = (torch.randn(B, T, C, generator=g).to(cuda).to(torch.bfloat16) for _ in range(3))
    with torch.no_grad():
        o1 = flash_attn(q, k, v, H, True, 0.1, 77)
        _, _, keep = _C.flash_attn_fwd(q, k, v, H, True, 0.1, 77, False)
    assert keep.numel() == 0
    o2 = flash_attn(q.clone().requires_grad_(True), k, v, H, True, 0.1, 77)
    assert torch.equal(o1, o2.detach())
