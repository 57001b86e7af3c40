"""Plain-PyTorch reference implementations of every fused op.

These are (a) the CPU execution path (tests, gloo plumbing runs) and (b) the numerics oracle the
HIP kernels are tested against. Math follows HF PyTorch BERT
([dep: transformers/models/bert/modeling_bert.py]) which is what the reference's TF model computes
(``scripts/train.py:117``): post-LN residual blocks, exact-erf GELU, additive key-padding mask.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from .rng import keep_mask


def dropout(x: torch.Tensor, p: float, seed: int, training: bool = True) -> torch.Tensor:
    if not training or p <= 0.0:
        return x
    m = keep_mask(seed, x.shape, p, device=x.device)
    return x * m.to(x.dtype) * (1.0 / (1.0 - p))


def embed_ln(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b,
             eps: float, p: float, seed: int, training: bool) -> torch.Tensor:
    """``dropout(LN(word[ids] + pos[pos_ids] + type[tt]))`` (modeling_bert.py BertEmbeddings)."""
    h = F.embedding(input_ids, word_w) + F.embedding(position_ids, pos_w)
    if type_w is not None:
        h = h + F.embedding(token_type_ids, type_w)
    h = F.layer_norm(h.float(), (h.shape[-1],), ln_w.float(), ln_b.float(), eps).to(word_w.dtype)
    return dropout(h, p, seed, training)


def linear(x, w, b):
    return F.linear(x, w, b)


def gelu(x):
    return F.gelu(x.float(), approximate="none").to(x.dtype)


def linear_gelu(x, w, b):
    return gelu(F.linear(x, w, b))


def linear_dropout_residual(x, w, b, residual, p: float, seed: int, training: bool):
    """``dropout(x Wᵀ + b) + residual`` rounded ONCE to the output dtype (fp32 product and sum), as the HIP epilogues
    compute it (gemm_common.h / gemm.hip: bf16(fma(y, keep · scale, residual)) with y = bf16(x Wᵀ + b))."""
    y = F.linear(x, w, b)
    if not training or p <= 0.0:
        return y + residual
    k = keep_mask(seed, y.shape, p, device=y.device).to(torch.float32) * (1.0 / (1.0 - p))
    return torch.addcmul(residual.float(), y.float(), k).to(y.dtype)


def layer_norm(x, w, b, eps: float):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def key_mask_bias(attention_mask: Optional[torch.Tensor], dtype=torch.float32) -> Optional[torch.Tensor]:
    """[B,S] 0/1 mask -> additive fp32 bias [B,S] (0 keep, -inf-like mask)."""
    if attention_mask is None:
        return None
    return (1.0 - attention_mask.to(torch.float32)) * torch.finfo(torch.float32).min


def attention(qkv: torch.Tensor, mask_bias: Optional[torch.Tensor], batch: int, seq: int, heads: int,
              p: float, seed: int, training: bool) -> torch.Tensor:
    """Self-attention over a packed ``[B*S, 3H]`` QKV tensor -> ``[B*S, H]`` context.

    Dropout on the probabilities: row ``(b*heads + h)*S + i``, column ``j`` of the site's [rows, S] view (ops/rng.py).
    """
    H3 = qkv.shape[-1]
    H = H3 // 3
    d = H // heads
    x = qkv.view(batch, seq, 3, heads, d).permute(2, 0, 3, 1, 4).float()  # [3,B,h,S,d]
    q, k, v = x[0], x[1], x[2]
    s = torch.matmul(q, k.transpose(-1, -2)) * (1.0 / math.sqrt(d))
    if mask_bias is not None:
        s = s + mask_bias.view(batch, 1, 1, seq).float()
    pr = torch.softmax(s, dim=-1)
    pr = dropout(pr, p, seed, training)
    o = torch.matmul(pr, v)  # [B,h,S,d]
    return o.permute(0, 2, 1, 3).reshape(batch * seq, H).to(qkv.dtype)


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """SparseCategoricalCrossentropy(from_logits=True), SUM_OVER_BATCH_SIZE (``scripts/train.py:118``)."""
    return F.cross_entropy(logits.float(), labels.long())


def accuracy_count(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    return (logits.argmax(dim=-1) == labels.long()).sum()


def cls_head(x, w1, b1, w2, b2, act: str, p_in: float, seed_in: int, p: float, seed: int, training: bool):
    """Sequence-classification head on the first-token rows ``x`` [B, H] -> logits [B, C]:
    ``W2·dropout(act(W1·dropout_in(x) + b1)) + b2`` (HF BertPooler + classifier, RobertaClassificationHead,
    DistilBERT pre_classifier; act = "tanh" | "relu")."""
    x = dropout(x, p_in, seed_in, training)
    h = F.linear(x, w1, b1)
    h = torch.tanh(h) if act == "tanh" else torch.relu(h)
    h = dropout(h, p, seed, training)
    return F.linear(h, w2, b2)


def mlm_head(h2d, labels, w1, b1, ln_w, ln_b, eps: float, wemb, bias, vocab: int):
    """RoBERTa LM head on the masked positions (labels != -100) of ``h2d`` [T, H]: ``LN(gelu(x W1ᵀ + b1))`` ->
    tied decoder (``wemb[:vocab]``, ``bias[:vocab]``) -> mean CE. Returns (loss, logits [n_masked, vocab])."""
    sel = labels.ne(-100).nonzero(as_tuple=True)[0]
    x = h2d.index_select(0, sel)
    x = layer_norm(linear_gelu(x, w1, b1), ln_w, ln_b, eps)
    logits = F.linear(x, wemb[:vocab], bias[:vocab])
    return cross_entropy(logits, labels.index_select(0, sel)), logits
