"""Op dispatch: one API, two implementations.

* CUDA (=HIP on ROCm) tensors -> hand-written gfx950 kernels in ``csrc/kernels`` via
  :mod:`.hip` (custom autograd Functions). If the compiled extension is missing on a GPU box this
  raises — there is no silent eager fallback.
* fp32 GPU tensors (``--dtype fp32``, the reference's own precision) -> :mod:`.hip32` (fp32 kernels in
  ``csrc/kernels/fp32.hip`` + split-product MFMA GEMMs).
* CPU tensors -> :mod:`.reference` (plain torch; also the numerics oracle for the kernel tests).

``HSD_OPS=torch`` forces the reference path on GPU (only for A/B measurements of the kernels); ``HSD_FP32_OPS=torch``
does so for fp32 tensors only.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import reference as _ref

_FORCE_TORCH = os.environ.get("HSD_OPS", "").lower() == "torch"
_FP32_TORCH = os.environ.get("HSD_FP32_OPS", "").lower() == "torch"


def _hip(x: torch.Tensor) -> bool:
    # bf16 / fp8 steps: the HIP kernels of ops/hip.py
    return x.is_cuda and not _FORCE_TORCH and x.dtype != torch.float32


def _hip32(x: torch.Tensor) -> bool:
    # fp32 steps (``--dtype fp32``, the reference's own precision: scripts/train.py:113-123 has no mixed-precision
    # policy): the fp32 kernels of ops/hip32.py
    return x.is_cuda and not _FORCE_TORCH and not _FP32_TORCH and x.dtype == torch.float32


def _hipmod():
    from . import hip  # noqa: WPS433 (lazy: imports the compiled extension)

    return hip


def _hip32mod():
    from . import hip32  # noqa: WPS433

    return hip32


def key_mask_bias(attention_mask: Optional[torch.Tensor]):
    if attention_mask is not None and attention_mask.is_cuda and not _FORCE_TORCH and \
            attention_mask.dtype in (torch.int64, torch.int32):
        return _hipmod().key_mask_bias(attention_mask)
    return _ref.key_mask_bias(attention_mask)


def dropout(x: torch.Tensor, p: float, seed: int):
    if p <= 0.0:
        return x
    if _hip(x):
        return _hipmod().dropout(x, p, seed)
    if _hip32(x):
        return _hip32mod().dropout(x, p, seed)
    return _ref.dropout(x, p, seed, True)


def embed_ln(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b, eps, p, seed,
             pos_is_arange=False, q8_for=None):
    if _hip(word_w):
        return _hipmod().embed_ln(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b,
                                  eps, p, seed, pos_is_arange, q8_for)
    if _hip32(word_w) and word_w.shape[1] % 4 == 0 and word_w.shape[1] <= 1024:
        return _hip32mod().embed_ln(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b,
                                    eps, p, seed)
    return _ref.embed_ln(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b, eps, p, seed,
                         p > 0)


def linear(x, w, b):
    if _hip(x):
        return _hipmod().linear(x, w, b)
    if _hip32(x):
        return _hip32mod().linear(x, w, b)
    return _ref.linear(x, w, b)


def linear_gelu(x, w, b):
    if _hip(x):
        return _hipmod().linear_gelu(x, w, b)
    if _hip32(x):
        return _hip32mod().linear_gelu(x, w, b)
    return _ref.linear_gelu(x, w, b)


def layer_norm(x, w, b, eps):
    if _hip(x):
        return _hipmod().layer_norm(x, w, b, eps)
    if _hip32(x) and x.shape[-1] % 4 == 0 and x.shape[-1] <= 1024:
        return _hip32mod().layer_norm(x, w, b, eps)
    return _ref.layer_norm(x, w, b, eps)


def dense_residual_ln(x, w, b, residual, ln_w, ln_b, eps, p, seed):
    """``LN(dropout(x Wᵀ + b) + residual)`` — the post-LN block tail."""
    if _hip(x):
        return _hipmod().dense_residual_ln(x, w, b, residual, ln_w, ln_b, eps, p, seed)
    if _hip32(x) and w.shape[0] % 4 == 0 and w.shape[0] <= 1024:
        return _hip32mod().dense_residual_ln(x, w, b, residual, ln_w, ln_b, eps, p, seed)
    return _ref.layer_norm(_ref.linear_dropout_residual(x, w, b, residual, p, seed, p > 0), ln_w, ln_b, eps)


def attn_block(h, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, eps, mask_bias, batch, seq, heads, p_attn, seed_attn,
               p_hidden, seed_hidden, q8_next=None):
    """Self-attention sub-block: ``LN(dropout(attn(h Wqkvᵀ + b) Woᵀ + bo) + h)``. ``q8_next``: the weight of the
    GEMM that consumes the output (HIP fp8 path: the LayerNorm writes its fp8 input copy)."""
    if _hip(h) and h.dtype == torch.bfloat16 and qkv_w.shape[0] == 3 * heads * 64:
        return _hipmod().attn_block(h, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, eps, mask_bias, batch, seq, heads,
                                    p_attn, seed_attn, p_hidden, seed_hidden, q8_next)
    if _hip32(h) and _hip32mod().attn_block_ok(h, qkv_w, seq, heads):
        return _hip32mod().attn_block(h, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, eps, mask_bias, batch, seq, heads,
                                      p_attn, seed_attn, p_hidden, seed_hidden)
    qkv = linear(h, qkv_w, qkv_b)
    ctx = attention(qkv, mask_bias, batch, seq, heads, p_attn, seed_attn)
    return dense_residual_ln(ctx, out_w, out_b, h, ln_w, ln_b, eps, p_hidden, seed_hidden)


def ffn_block(h, w1, b1, w2, b2, ln_w, ln_b, eps, p, seed, q8_next=None):
    """Feed-forward sub-block: ``LN(dropout(gelu(h W1ᵀ + b1) W2ᵀ + b2) + h)``."""
    if _hip(h) and h.dtype == torch.bfloat16:
        return _hipmod().ffn_block(h, w1, b1, w2, b2, ln_w, ln_b, eps, p, seed, q8_next)
    if _hip32(h) and _hip32mod().ffn_block_ok(h, w1):
        return _hip32mod().ffn_block(h, w1, b1, w2, b2, ln_w, ln_b, eps, p, seed)
    a = linear_gelu(h, w1, b1)
    return dense_residual_ln(a, w2, b2, h, ln_w, ln_b, eps, p, seed)


def attention(qkv, mask_bias, batch, seq, heads, p, seed):
    if _hip(qkv):
        return _hipmod().attention(qkv, mask_bias, batch, seq, heads, p, seed)
    if _hip32(qkv):
        return _hip32mod().attention(qkv, mask_bias, batch, seq, heads, p, seed)
    return _ref.attention(qkv, mask_bias, batch, seq, heads, p, seed, p > 0)


def hip_active(device) -> bool:
    """True when tensors on ``device`` run the HIP kernels (not the reference ops)."""
    return torch.device(device).type == "cuda" and not _FORCE_TORCH


def set_fp8(on: bool, grad_fmt: str = "e4m3") -> None:
    """Route the encoder's forward / dgrad GEMMs through the fp8 kernel (weights need fp8 copies:
    ``FlatParamStore(..., fp8=True)``)."""
    _hipmod().set_fp8(on, grad_fmt)


def join_side_streams() -> None:
    """Order the current stream after the wgrad side stream (no-op on CPU / reference ops)."""
    if torch.cuda.is_available() and not _FORCE_TORCH:
        _hipmod().join_side_streams()


def cross_entropy(logits, labels):
    """Mean CE over non-ignored labels. On the HIP path the fused kernel also counts argmax hits; the count
    rides on the loss tensor (``loss._hsd_correct``) so metrics need no second pass over the logits."""
    if _hip(logits):
        loss, correct = _hipmod().cross_entropy(logits, labels)
        loss._hsd_correct = correct
        return loss
    return _ref.cross_entropy(logits, labels)


def cls_head(h, w1, b1, w2, b2, labels, act: str, p_in: float, seed_in: int, p: float, seed: int):
    """Classification head on the first token of ``h`` [B, S, H] (+ the loss when ``labels`` is given).

    Returns ``logits`` without labels, else ``(loss, logits)`` with the argmax-hit count on ``loss._hsd_correct``
    and the fused {mean loss, hits, rows, loss sum} on ``loss._hsd_stats`` (HIP path). On GPUs the dense layer runs on gemm2 and everything after it (activation, dropout, classifier, CE,
    accuracy) in one fused kernel per direction (csrc/kernels/cls_head.hip); the first-token rows are read in place
    (no gather copy) and their gradient is written straight into the zeroed ``dh`` rows."""
    if _hip(h) and labels is not None and _hipmod().cls_head_ok(h, w1, w2):
        loss, logits, stats = _hipmod().cls_head(h, w1, b1, w2, b2, labels, act, p_in, seed_in, p, seed)
        loss._hsd_correct = stats[1]
        loss._hsd_stats = stats  # {mean loss, hits, rows, loss sum}: the metric meter folds these lazily
        return loss, logits
    if _hip32(h) and labels is not None and _hip32mod().cls_head_ok(h, w1, w2):
        loss, logits, stats = _hip32mod().cls_head(h, w1, b1, w2, b2, labels, act, p_in, seed_in, p, seed)
        loss._hsd_correct = stats[1]
        loss._hsd_stats = stats
        return loss, logits
    x = h[:, 0].contiguous()
    if _hip(h) or _hip32(h):
        x = dropout(x, p_in, seed_in)
        y = linear(x, w1, b1)
        y = torch.tanh(y) if act == "tanh" else torch.relu(y)
        y = dropout(y, p, seed)
        logits = linear(y, w2, b2)
    else:
        logits = _ref.cls_head(x, w1, b1, w2, b2, act, p_in, seed_in, p, seed, True)
    if labels is None:
        return logits
    return cross_entropy(logits, labels), logits


def mlm_head(h2d, labels, w1, b1, ln_w, ln_b, eps, wemb, bias, vocab):
    """Masked-LM head (RoBERTa) on the masked rows of ``h2d`` -> (loss, logits over the real vocabulary).

    GPU: every GEMM on gemm2 (dense + GELU epilogue, LN kernel, the tied decoder over the 256-padded vocabulary, its
    dgrad reading the embedding table directly and the embedding-table weight gradient), the chunked-vocabulary CE
    kernel; the argmax-hit count rides on ``loss._hsd_correct``."""
    if _hip(h2d) and h2d.dtype == torch.bfloat16 and _hipmod().mlm_head_ok(h2d, w1, wemb):
        loss, logits, correct = _hipmod().mlm_head(h2d, labels, w1, b1, ln_w, ln_b, eps, wemb, bias, vocab)
        loss._hsd_correct = correct
        return loss, logits
    if _hip(h2d):
        sel = labels.ne(-100).nonzero(as_tuple=True)[0]
        x = h2d.index_select(0, sel)
        x = layer_norm(linear_gelu(x, w1, b1), ln_w, ln_b, eps)
        logits = linear(x, wemb[:vocab], bias[:vocab])
        return cross_entropy(logits, labels.index_select(0, sel)), logits
    return _ref.mlm_head(h2d, labels, w1, b1, ln_w, ln_b, eps, wemb, bias, vocab)


def accuracy_count(logits, labels):
    return _ref.accuracy_count(logits, labels)
