"""BERT-base (110 M) pre-training model — BASELINE config #3.

12 layers, hidden 768, 12 heads, FFN 3072, max 512 positions, vocab 30522,
GELU(erf), post-LN; heads: masked-LM (transform + tied decoder) and
next-sentence prediction. Random init (std 0.02).

MI355X path: every LayerNorm is the hand-written kernel; the MLM head runs
only on the masked positions (gathered first: ~15 % of tokens), and its
vocab cross-entropy is the fused kernel on bf16 logits; attention is our MFMA
flash-attention kernel (``ops/attention.py``; ``scaled_dot_product_attention``
when a padding mask is given or with ``fused=False``).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn
from torch.nn import functional as F

from ..ops.attention import attn_supported, flash_attn_qkv
from ..ops.embedding import FusedEmbedding
from ..ops.linear import FusedLinear, LinearWeightPrep, fused_mlp_gelu, packed_linear
from ..ops.lm_head import lm_head_cross_entropy, padded_vocab
from ..ops.dropout import dropout_add
from ..ops import layernorm as ln_mod
from ..ops.layernorm import FusedLayerNorm, dropout_add_layer_norm


def _plain_dropout_add(x, residual, p, training):
    return residual + F.dropout(x, p, training)


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    dropout: float = 0.1
    eps: float = 1e-12
    fused: bool = True


def _ln(cfg, d):
    return FusedLayerNorm(d, eps=cfg.eps) if cfg.fused else nn.LayerNorm(d, eps=cfg.eps)


class BertSelfAttention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.heads = cfg.heads
        lin = FusedLinear if cfg.fused else nn.Linear
        self.query = lin(cfg.hidden, cfg.hidden)
        self.key = lin(cfg.hidden, cfg.hidden)
        self.value = lin(cfg.hidden, cfg.hidden)
        self.dropout = cfg.dropout
        self.fused = cfg.fused

    def forward(self, x, mask):
        B, T, C = x.shape
        h = self.heads
        if self.fused and mask is None:
            # query / key / value as one packed GEMM (one dgrad GEMM, no
            # per-projection gradient adds) feeding the packed MFMA flash attention
            qkv = packed_linear(x, (self.query, self.key, self.value))
            if attn_supported(qkv[..., :C], h):
                return flash_attn_qkv(qkv, h, causal=False, dropout_p=self.dropout if self.training else 0.0)
            q, k, v = qkv.split(C, dim=2)
            return F.scaled_dot_product_attention(
                q.view(B, T, h, C // h).transpose(1, 2), k.view(B, T, h, C // h).transpose(1, 2),
                v.view(B, T, h, C // h).transpose(1, 2),
                dropout_p=self.dropout if self.training else 0.0).transpose(1, 2).reshape(B, T, C)

        def split(t):
            return t.view(B, T, h, C // h).transpose(1, 2)

        y = F.scaled_dot_product_attention(split(self.query(x)), split(self.key(x)), split(self.value(x)),
                                           attn_mask=mask, dropout_p=self.dropout if self.training else 0.0)
        return y.transpose(1, 2).reshape(B, T, C)


class BertLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.attention = BertSelfAttention(cfg)
        lin = FusedLinear if cfg.fused else nn.Linear
        self.attn_out = lin(cfg.hidden, cfg.hidden)
        self.attn_ln = _ln(cfg, cfg.hidden)
        self.intermediate = lin(cfg.hidden, cfg.intermediate)
        self.output = lin(cfg.intermediate, cfg.hidden)
        self.out_ln = _ln(cfg, cfg.hidden)
        self.p = cfg.dropout
        self._dadd = dropout_add if cfg.fused else _plain_dropout_add

    def forward(self, x, mask, x_res=None, dual_out: bool = False):
        """``x_res``: an alias of ``x`` for the residual add (the previous
        layer's dual-output LN), ``dual_out``: return (y, alias of y). With the
        fused LNs every post-LN output's two gradients (next sublayer + its
        residual add) are summed inside the LN backward instead of by an add."""
        dual = isinstance(self.attn_ln, FusedLayerNorm)
        x_res = x if x_res is None else x_res
        fuse = dual and ln_mod.FUSE_DADD_LN
        if fuse:  # residual dropout-add inside the LayerNorm kernels (ops.layernorm.dropout_add_layer_norm)
            x, xa = dropout_add_layer_norm(self.attn_out(self.attention(x, mask)), x_res, self.attn_ln, self.p,
                                           self.training, 2)
        else:
            h = self._dadd(self.attn_out(self.attention(x, mask)), x_res, self.p, self.training)
            x, xa = self.attn_ln.forward_dual_out(h) if dual else (self.attn_ln(h), None)
        if isinstance(self.intermediate, FusedLinear):
            # one node: GELU in the first GEMM's epilogue, its backward in the second's dgrad epilogue
            o = fused_mlp_gelu(x, self.intermediate, self.output, "none")
        else:
            o = self.output(F.gelu(self.intermediate(x)))
        if fuse:
            if dual_out:
                return dropout_add_layer_norm(o, xa, self.out_ln, self.p, self.training, 2)
            return dropout_add_layer_norm(o, xa, self.out_ln, self.p, self.training, 0)
        h = self._dadd(o, x if xa is None else xa, self.p, self.training)
        if dual_out and dual:
            return self.out_ln.forward_dual_out(h)
        y = self.out_ln(h)
        return (y, None) if dual_out else y


class BertForPreTraining(nn.Module):
    def __init__(self, cfg: BertConfig = BertConfig()):
        super().__init__()
        self.cfg = cfg
        self.word_embeddings = (FusedEmbedding if cfg.fused else nn.Embedding)(cfg.vocab_size, cfg.hidden)
        self.position_embeddings = (FusedEmbedding if cfg.fused else nn.Embedding)(cfg.max_position, cfg.hidden)
        self.token_type_embeddings = (FusedEmbedding if cfg.fused else nn.Embedding)(cfg.type_vocab, cfg.hidden)
        self.emb_ln = _ln(cfg, cfg.hidden)
        self.emb_drop = nn.Dropout(cfg.dropout)
        self.layers = nn.ModuleList([BertLayer(cfg) for _ in range(cfg.layers)])
        self.pooler = nn.Linear(cfg.hidden, cfg.hidden)
        self.mlm_transform = (FusedLinear if cfg.fused else nn.Linear)(cfg.hidden, cfg.hidden)
        self.mlm_ln = _ln(cfg, cfg.hidden)
        self.mlm_bias = nn.Parameter(torch.zeros(cfg.vocab_size))
        self.nsp = nn.Linear(cfg.hidden, 2)
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, 0.0, 0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, mlm_labels=None, nsp_labels=None,
                mlm_positions=None):
        """``mlm_labels``: either [B, T] with -100 for unmasked tokens, or — with
        ``mlm_positions`` [B, P] (fixed predictions per sequence, no host sync) —
        the [B, P] label ids of those positions."""
        B, T = input_ids.shape
        if self.cfg.fused and input_ids.is_cuda:
            # bf16 W / Wᵀ of every Linear, packed QKV and the padded MLM head: one launch per optimizer step
            LinearWeightPrep.attach(
                self, packed=[(l.attention.query.weight, l.attention.key.weight, l.attention.value.weight)
                              for l in self.layers],
                heads={self.word_embeddings.weight: padded_vocab(self.cfg.vocab_size)})
        pos = torch.arange(T, device=input_ids.device)
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos) + self.token_type_embeddings(
            token_type_ids)
        x = self.emb_drop(self.emb_ln(x))
        mask = None
        if attention_mask is not None:
            mask = attention_mask[:, None, None, :].to(torch.bool)
        xa = None
        for i, layer in enumerate(self.layers):
            if i + 1 < len(self.layers):
                x, xa = layer(x, mask, xa, dual_out=True)
            else:
                x = layer(x, mask, xa)
        pooled = torch.tanh(self.pooler(x[:, 0]))
        nsp_logits = self.nsp(pooled)
        if mlm_labels is None:
            return x, nsp_logits
        # MLM head on masked positions only
        if mlm_positions is not None:
            sel = (mlm_positions + torch.arange(B, device=x.device)[:, None] * T).reshape(-1)
            tgt = mlm_labels.reshape(-1)
        else:
            flat_labels = mlm_labels.reshape(-1)
            sel = (flat_labels != -100).nonzero(as_tuple=True)[0]  # host sync: prefer mlm_positions
            tgt = flat_labels.index_select(0, sel)
        h = x.reshape(B * T, -1).index_select(0, sel)
        if isinstance(self.mlm_transform, FusedLinear):
            h = self.mlm_ln(self.mlm_transform.forward_gelu(h))
        else:
            h = self.mlm_ln(F.gelu(self.mlm_transform(h)))
        if self.cfg.fused:
            mlm = lm_head_cross_entropy(h, self.word_embeddings.weight, self.mlm_bias, tgt)
        else:
            mlm = F.cross_entropy(F.linear(h, self.word_embeddings.weight, self.mlm_bias).float(), tgt)
        loss = mlm
        if nsp_labels is not None:
            loss = loss + F.cross_entropy(nsp_logits.float(), nsp_labels)
        return loss


def bert_base(**kw) -> BertForPreTraining:
    return BertForPreTraining(BertConfig(**kw))
