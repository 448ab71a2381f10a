"""GPT-2 small (124 M) — BASELINE config #5 (DDP + gradient accumulation + bf16 AMP).

12 layers, d_model 768, 12 heads, context 1024, vocab 50257, GELU(tanh), pre-LN,
tied LM head. Random init (std 0.02, residual projections scaled by
1/sqrt(2·n_layer)). Parameter names follow the common GPT-2 layout
(wte, wpe, h.N.ln_1, h.N.attn.c_attn, ...).

MI355X path: LayerNorm = hand-written kernel (bf16 activations, fp32 stats),
attention = our MFMA flash-attention kernels on the packed qkv projection
(causal, in-kernel dropout; ``ops/attention.py``), loss = fused vocab
cross-entropy straight from bf16 logits. ``fused=False`` is the stock path
(``scaled_dot_product_attention``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
from torch import nn
from torch.nn import functional as F

from ..ops.attention import attn_supported, flash_attn_qkv
from ..ops.cross_entropy import fused_cross_entropy
from ..ops.embedding import FusedEmbedding
from ..ops.linear import FusedLinear, LinearWeightPrep, fused_mlp_gelu
from ..ops.lm_head import lm_head_cross_entropy, padded_vocab
from ..ops.dropout import dropout_add
from ..ops import layernorm as ln_mod
from ..ops.layernorm import FusedLayerNorm, dropout_add_layer_norm


def _plain_dropout_add(x, residual, p, training):
    return residual + F.dropout(x, p, training)


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    dropout: float = 0.1
    fused: bool = True


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.n_head = cfg.n_head
        lin = FusedLinear if cfg.fused else nn.Linear
        self.c_attn = lin(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = lin(cfg.n_embd, cfg.n_embd)
        self.dropout = cfg.dropout
        self.fused = cfg.fused

    def forward(self, x):
        B, T, C = x.shape
        qkv = self.c_attn(x)
        if self.fused and attn_supported(qkv[..., :C], self.n_head):
            # MFMA flash attention on the packed projection: no head transposes,
            # dq/dk/dv written straight into one packed gradient
            y = flash_attn_qkv(qkv, self.n_head, causal=True, dropout_p=self.dropout if self.training else 0.0)
            return self.c_proj(y)
        q, k, v = qkv.split(C, dim=2)
        h = self.n_head
        q = q.view(B, T, h, C // h).transpose(1, 2)
        k = k.view(B, T, h, C // h).transpose(1, 2)
        v = v.view(B, T, h, C // h).transpose(1, 2)
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout if self.training else 0.0, is_causal=True)
        y = y.transpose(1, 2).contiguous().view(B, T, C)
        return self.c_proj(y)  # residual dropout is fused with the add in Block


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        lin = FusedLinear if cfg.fused else nn.Linear
        self.c_fc = lin(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = lin(4 * cfg.n_embd, cfg.n_embd)

    def forward(self, x):
        if isinstance(self.c_fc, FusedLinear):
            # one node: GELU in c_fc's GEMM epilogue, its backward in c_proj's dgrad epilogue
            return fused_mlp_gelu(x, self.c_fc, self.c_proj, "tanh")
        return self.c_proj(F.gelu(self.c_fc(x), approximate="tanh"))


def _ln(cfg, d):
    return FusedLayerNorm(d) if cfg.fused else nn.LayerNorm(d)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = _ln(cfg, cfg.n_embd)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = _ln(cfg, cfg.n_embd)
        self.mlp = MLP(cfg)
        self.p = cfg.dropout
        self._dadd = dropout_add if cfg.fused else _plain_dropout_add

    def forward_pending(self, x, pending=None):
        """The fused block: ``pending`` is the previous block's MLP output whose
        residual dropout-add runs inside this block's first LayerNorm kernel
        (ops.layernorm.dropout_add_layer_norm); returns (this block's MLP
        output, the residual stream before its dropout-add)."""
        if pending is None:
            h, x = self.ln_1.forward_dual(x)
        else:
            h, x = dropout_add_layer_norm(pending, x, self.ln_1, self.p, self.training, 1)
        h, x = dropout_add_layer_norm(self.attn(h), x, self.ln_2, self.p, self.training, 1)
        return self.mlp(h), x

    def forward(self, x):
        if isinstance(self.ln_1, FusedLayerNorm):
            # dual-output LN: the residual stream's two gradients (branch + skip)
            # are summed inside the LN backward kernel, not by an fp32 add
            h, x = self.ln_1.forward_dual(x)
            x = self._dadd(self.attn(h), x, self.p, self.training)
            h, x = self.ln_2.forward_dual(x)
            return self._dadd(self.mlp(h), x, self.p, self.training)
        x = self._dadd(self.attn(self.ln_1(x)), x, self.p, self.training)
        return self._dadd(self.mlp(self.ln_2(x)), x, self.p, self.training)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config = GPT2Config()):
        super().__init__()
        self.cfg = cfg
        self.wte = (FusedEmbedding if cfg.fused else nn.Embedding)(cfg.vocab_size, cfg.n_embd)
        self.wpe = (FusedEmbedding if cfg.fused else nn.Embedding)(cfg.n_positions, cfg.n_embd)
        self.drop = nn.Dropout(cfg.dropout)
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = _ln(cfg, cfg.n_embd)
        self.apply(self._init)
        for n, p in self.named_parameters():
            if n.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * cfg.n_layer))

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, 0.02)

    def forward(self, idx, targets=None):
        B, T = idx.shape
        if self.cfg.fused and idx.is_cuda:
            # bf16 W / Wᵀ of every Linear and the padded tied head: one launch per optimizer step
            LinearWeightPrep.attach(self, heads={self.wte.weight: padded_vocab(self.cfg.vocab_size)})
        pos = torch.arange(T, device=idx.device)
        x = self.drop(self.wte(idx) + self.wpe(pos))
        if self.cfg.fused and ln_mod.FUSE_DADD_LN and isinstance(self.ln_f, FusedLayerNorm) and x.is_cuda:
            pending = None
            for blk in self.h:
                pending, x = blk.forward_pending(x, pending)
            x = dropout_add_layer_norm(pending, x, self.ln_f, self.cfg.dropout, self.training, 0)
        else:
            for blk in self.h:
                x = blk(x)
            x = self.ln_f(x)
        if targets is not None and self.cfg.fused:
            # tied head + cross-entropy as one node on our GEMMs (no logits returned)
            return lm_head_cross_entropy(x, self.wte.weight, None, targets)
        logits = F.linear(x, self.wte.weight)  # tied head
        if targets is None:
            return logits
        flat = logits.view(B * T, -1)
        if self.cfg.fused:
            loss = fused_cross_entropy(flat, targets.reshape(-1))
        else:
            loss = F.cross_entropy(flat.float(), targets.reshape(-1))
        return loss


def gpt2_small(**kw) -> GPT2:
    return GPT2(GPT2Config(**kw))
