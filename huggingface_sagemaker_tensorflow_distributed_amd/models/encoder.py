"""Post-LN transformer encoder shared by BERT, RoBERTa and DistilBERT.

The reference trains ``TFAutoModelForSequenceClassification`` (``scripts/train.py:117``); its math is
HF BERT's ([dep: transformers/models/bert/modeling_bert.py]):

    qkv  = X Wqkvᵀ + b           (three Linears in HF; one N=3H GEMM here, split only at save time)
    ctx  = softmax(QKᵀ/√d + mask) V   (+ dropout on the probabilities)
    h1   = LN(dropout(ctx Woᵀ + bo) + X)
    h2   = LN(dropout(gelu(h1 W1ᵀ + b1) W2ᵀ + b2) + h1)

Parameters are stored FUSED (``qkv_weight`` = [3H, H]) so the QKV projection is one MFMA GEMM; the
HF key names are produced by :mod:`..models.hf_io` from :meth:`hf_names`.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..ops.rng import DropoutSeeds
from .config import ModelConfig


def _param(*shape) -> nn.Parameter:
    return nn.Parameter(torch.empty(*shape))


class EncoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        H, I = cfg.hidden_size, cfg.intermediate_size
        self.cfg = cfg
        # declaration order == forward use order (the flat store reverses it for backward bucketing)
        self.qkv_weight = _param(3 * H, H)
        self.qkv_bias = _param(3 * H)
        self.attn_out_weight = _param(H, H)
        self.attn_out_bias = _param(H)
        self.ln1_weight = _param(H)
        self.ln1_bias = _param(H)
        self.ffn1_weight = _param(I, H)
        self.ffn1_bias = _param(I)
        self.ffn2_weight = _param(H, I)
        self.ffn2_bias = _param(H)
        self.ln2_weight = _param(H)
        self.ln2_bias = _param(H)

    def forward(self, h: torch.Tensor, mask_bias: Optional[torch.Tensor], batch: int, seq: int,
                rng: DropoutSeeds, training: bool, next_qkv: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``next_qkv``: the next layer's QKV weight (fp8 path: this layer's last LayerNorm quantises for it)."""
        c = self.cfg
        p_h = c.hidden_dropout_prob if training else 0.0
        p_a = c.attention_probs_dropout_prob if training else 0.0
        seed_a = rng.next() if p_a else 0
        seed_h1 = rng.next() if p_h else 0
        h1 = ops.attn_block(h, self.qkv_weight, self.qkv_bias, self.attn_out_weight, self.attn_out_bias,
                            self.ln1_weight, self.ln1_bias, c.layer_norm_eps, mask_bias, batch, seq,
                            c.num_attention_heads, p_a, seed_a, p_h, seed_h1, q8_next=self.ffn1_weight)
        seed_h2 = rng.next() if p_h else 0
        return ops.ffn_block(h1, self.ffn1_weight, self.ffn1_bias, self.ffn2_weight, self.ffn2_bias,
                             self.ln2_weight, self.ln2_bias, c.layer_norm_eps, p_h, seed_h2, q8_next=next_qkv)


# name tables: internal name -> list of (hf suffix, row-slice or None)
_BERT_LAYER_NAMES = {
    "qkv_weight": ("attention.self.{}.weight", ("query", "key", "value")),
    "qkv_bias": ("attention.self.{}.bias", ("query", "key", "value")),
    "attn_out_weight": ("attention.output.dense.weight", None),
    "attn_out_bias": ("attention.output.dense.bias", None),
    "ln1_weight": ("attention.output.LayerNorm.weight", None),
    "ln1_bias": ("attention.output.LayerNorm.bias", None),
    "ffn1_weight": ("intermediate.dense.weight", None),
    "ffn1_bias": ("intermediate.dense.bias", None),
    "ffn2_weight": ("output.dense.weight", None),
    "ffn2_bias": ("output.dense.bias", None),
    "ln2_weight": ("output.LayerNorm.weight", None),
    "ln2_bias": ("output.LayerNorm.bias", None),
}
_DISTIL_LAYER_NAMES = {
    "qkv_weight": ("attention.{}.weight", ("q_lin", "k_lin", "v_lin")),
    "qkv_bias": ("attention.{}.bias", ("q_lin", "k_lin", "v_lin")),
    "attn_out_weight": ("attention.out_lin.weight", None),
    "attn_out_bias": ("attention.out_lin.bias", None),
    "ln1_weight": ("sa_layer_norm.weight", None),
    "ln1_bias": ("sa_layer_norm.bias", None),
    "ffn1_weight": ("ffn.lin1.weight", None),
    "ffn1_bias": ("ffn.lin1.bias", None),
    "ffn2_weight": ("ffn.lin2.weight", None),
    "ffn2_bias": ("ffn.lin2.bias", None),
    "ln2_weight": ("output_layer_norm.weight", None),
    "ln2_bias": ("output_layer_norm.bias", None),
}


def layer_hf_names(layer_prefix: str, internal_prefix: str, distil: bool) -> Iterator[Tuple[str, str, Optional[int], int]]:
    """Yield ``(hf_key, internal_key, split_index, n_splits)``."""
    table = _DISTIL_LAYER_NAMES if distil else _BERT_LAYER_NAMES
    for iname, (fmt, parts) in table.items():
        if parts is None:
            yield layer_prefix + fmt, internal_prefix + iname, None, 1
        else:
            for i, part in enumerate(parts):
                yield layer_prefix + fmt.format(part), internal_prefix + iname, i, len(parts)
