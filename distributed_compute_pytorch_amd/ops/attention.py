"""Flash attention on the hand-written MFMA kernels (``csrc/kernels/attention.hip``).

Head dim 64, bf16 activations, fp32 softmax statistics, optional causal mask
and dropout on the attention probabilities (keep decisions hashed from a
counter in the forward and kept as bits, T²/8 bytes per head, for the
backward). Replaces
``scaled_dot_product_attention`` (PyTorch-ROCm's aotriton kernels) for
GPT-2-small and BERT-base.

* :func:`flash_attn` — q, k, v as [B, T, H*64] (any row stride: slices of a
  packed projection are read in place), output [B, T, H*64] — already the
  layout the output projection consumes (no head transposes).
* :func:`flash_attn_qkv` — packed [B, T, 3*H*64] input (GPT-2's ``c_attn``);
  the backward writes dq/dk/dv straight into one packed gradient (no cat).
"""
from __future__ import annotations

import torch

from .._ext import C as _C


def _seed() -> int:
    # from torch's CPU generator: torch.manual_seed makes runs reproducible
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


def attn_supported(x: torch.Tensor, heads: int) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 3
            and bool(_C.attn_ok(x.shape[1], x.shape[2], heads)))


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, heads, causal, p_drop, seed, keep_bits):
        o, lse, keep = _C.flash_attn_fwd(q, k, v, heads, causal, p_drop, seed, keep_bits)
        ctx.save_for_backward(q, k, v, o, lse, keep)
        ctx.cfg = (heads, causal, p_drop, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, keep = ctx.saved_tensors
        heads, causal, p_drop, seed = ctx.cfg
        do = do.contiguous()
        if do.dtype != torch.bfloat16:
            do = do.to(torch.bfloat16)
        dq, dk, dv = torch.empty_like(q, memory_format=torch.contiguous_format), torch.empty_like(
            k, memory_format=torch.contiguous_format), torch.empty_like(v, memory_format=torch.contiguous_format)
        _C.flash_attn_bwd(do, q, k, v, o, lse, keep, heads, causal, p_drop, seed, dq, dk, dv)
        return dq, dk, dv, None, None, None, None, None


class _FlashAttnQKVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, causal, p_drop, seed, keep_bits):
        C = qkv.shape[2] // 3
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        o, lse, keep = _C.flash_attn_fwd(q, k, v, heads, causal, p_drop, seed, keep_bits)
        ctx.save_for_backward(qkv, o, lse, keep)
        ctx.cfg = (heads, causal, p_drop, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, keep = ctx.saved_tensors
        heads, causal, p_drop, seed = ctx.cfg
        do = do.contiguous()
        if do.dtype != torch.bfloat16:
            do = do.to(torch.bfloat16)
        C = qkv.shape[2] // 3
        dqkv = torch.empty_like(qkv, memory_format=torch.contiguous_format)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        dq, dk, dv = dqkv[..., :C], dqkv[..., C:2 * C], dqkv[..., 2 * C:]
        _C.flash_attn_bwd(do, q, k, v, o, lse, keep, heads, causal, p_drop, seed, dq, dk, dv)
        return dqkv, None, None, None, None, None


def flash_attn(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int, causal: bool = False,
               dropout_p: float = 0.0, seed: int = None) -> torch.Tensor:
    """softmax(q kᵀ / 8 [+ causal mask]) → dropout(p) → · v, per head of 64."""
    return _FlashAttnFn.apply(q, k, v, heads, causal, float(dropout_p), _seed() if seed is None else int(seed),
                              _backward_will_run(q, k, v))


def flash_attn_qkv(qkv: torch.Tensor, heads: int, causal: bool = False, dropout_p: float = 0.0,
                   seed: int = None) -> torch.Tensor:
    return _FlashAttnQKVFn.apply(qkv, heads, causal, float(dropout_p), _seed() if seed is None else int(seed),
                                 _backward_will_run(qkv))


def _backward_will_run(*ts) -> bool:
    """Whether the forward must keep the dropout keep bits (T²/8 bytes per
    head) for a backward: grad mode on and some input requires grad."""
    return torch.is_grad_enabled() and any(t.requires_grad for t in ts)


def dropout_p_effective(p: float) -> float:
    """The dropout probability the kernels apply: ``p`` rounded to a multiple
    of 1/256 (byte thresholds, as FlashAttention-2 does); kept elements are
    scaled by 1 / (1 - dropout_p_effective(p))."""
    return int(p * 256.0 + 0.5) / 256.0


def flash_attn_keep_bits(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int, causal: bool,
                         dropout_p: float, seed: int) -> torch.Tensor:
    """The dropout keep decisions the forward stored for the backward, decoded
    to a bool [B, H, T, T] (test hook). Causal: entries above the diagonal are
    not stored (never read) and come back as False."""
    B, T = q.shape[0], q.shape[1]
    _, _, words = _C.flash_attn_fwd(q, k, v, heads, causal, float(dropout_p), int(seed))
    nblk = T // 64
    w = words.view(B * heads, nblk, 2, T).to(torch.int64) & 0xFFFFFFFF
    kk = torch.arange(64, device=q.device)
    # key 32kh + 8g + 4hh + e of a 64-key block: word half hh, bit 8e + 4kh + g
    hh, bit = (kk >> 2) & 1, 8 * (kk & 3) + 4 * ((kk >> 5) & 1) + ((kk >> 3) & 3)
    sel = w[:, :, hh, :]                                   # [BH, nblk, 64 keys, T queries]
    bits = (sel >> bit[None, None, :, None]) & 1
    m = bits.permute(0, 3, 1, 2).reshape(B, heads, T, T).bool()
    if causal:
        m &= torch.ones(T, T, dtype=torch.bool, device=q.device).tril()
    return m


def dropout_keep_mask(B: int, H: int, T: int, p: float, seed: int, device=None) -> torch.Tensor:
    """The kernels' dropout keep-mask [B, H, T, T] rebuilt with integer torch
    ops (test oracle). Per (query q, 64-key block k, lane half hh):
    x0 = fmix32(((q << 8) | (k << 1) | hh) ^ kbh), kbh = fmix32(s0 ^
    fmix32(bh·0x9E3779B1 + s1)) (murmur3 finaliser); word j (j < 8) is
    xorshift32 (13/17/5) applied j times to x0, XOR j·0x9E3779B9; key
    64k + 32(j >> 2) + 8(j & 3) + 4hh + e takes byte e of word j and is
    kept when that byte ≥ round(256·p)."""
    M = 0xFFFFFFFF
    dev = device or "cpu"

    def mul32(x, c):  # (x * c) mod 2^32 without int64 overflow
        lo, hi = x & 0xFFFF, x >> 16
        return ((lo * c) + (((hi * c) & 0xFFFF) << 16)) & M

    def fmix32(x):
        x = x ^ (x >> 16)
        x = mul32(x, 0x85EBCA6B)
        x = x ^ (x >> 13)
        x = mul32(x, 0xC2B2AE35)
        return x ^ (x >> 16)

    def xorshift32(x):
        x = x ^ ((x << 13) & M)
        x = x ^ (x >> 17)
        return x ^ ((x << 5) & M)

    nblk = T // 64
    s0, s1 = seed & M, (seed >> 32) & M
    i64 = dict(device=dev, dtype=torch.int64)
    bh = torch.arange(B * H, **i64)[:, None, None, None]
    qq = torch.arange(T, **i64)[None, :, None, None]
    kb = torch.arange(nblk, **i64)[None, None, :, None]
    hh = torch.arange(2, **i64)[None, None, None, :]
    kbh = fmix32(s0 ^ fmix32((mul32(bh, 0x9E3779B1) + s1) & M))
    x = fmix32(((qq << 8) | (kb << 1) | hh) ^ kbh)          # [BH, T, nblk, 2]
    words = []
    for j in range(8):
        words.append(x ^ ((j * 0x9E3779B9) & M))
        x = xorshift32(x)
    w = torch.stack(words, -1)                               # [BH, T, nblk, hh, j]
    e = torch.arange(4, **i64)
    r8 = (w[..., None] >> (8 * e)) & 0xFF                    # [BH, T, nblk, hh, j, e]
    thr = int(p * 256.0 + 0.5)
    keep = (r8 >= thr).reshape(B * H, T, nblk, 64)           # block offsets in (hh, j, e) order
    hv, jv, ev = torch.meshgrid(torch.arange(2), torch.arange(8), torch.arange(4), indexing="ij")
    off = (32 * (jv >> 2) + 8 * (jv & 3) + 4 * hv + ev).reshape(-1)
    inv = torch.empty_like(off)
    inv[off] = torch.arange(64)
    return keep[..., inv.to(keep.device)].reshape(B, H, T, T)
