"""BERT / RoBERTa / DistilBERT models with HF-identical checkpoint names.

Stands in for ``TFAutoModelForSequenceClassification.from_pretrained(name)``
(``scripts/train.py:117``, ``scripts/singe_node_train.py:43``): an encoder, the family's
sequence-classification head with a freshly initialised classifier, logits out. The RoBERTa MLM
model serves the ``roberta-large MLM`` north-star config (BASELINE.json configs[4]).

HF layout is produced by :meth:`hf_names`; internal storage fuses Q/K/V.
"""
from __future__ import annotations

import math
from typing import Dict, Iterator, Optional, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..ops.rng import DropoutSeeds
from .config import ModelConfig
from .encoder import EncoderLayer, _param, layer_hf_names


class Embeddings(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        H = cfg.hidden_size
        self.cfg = cfg
        self.word_embeddings = _param(cfg.vocab_size, H)
        self.position_embeddings = _param(cfg.max_position_embeddings, H)
        self.token_type_embeddings = _param(cfg.type_vocab_size, H) if cfg.type_vocab_size > 0 else None
        self.ln_weight = _param(H)
        self.ln_bias = _param(H)

    def position_ids(self, input_ids: torch.Tensor) -> torch.Tensor:
        B, S = input_ids.shape
        if self.cfg.model_type == "roberta":
            # HF create_position_ids_from_input_ids: padding_idx + cumsum over non-pad tokens
            pad = self.cfg.pad_token_id
            m = input_ids.ne(pad).int()
            return (torch.cumsum(m, dim=1).type_as(m) * m).long() + pad
        return self._cached("pos", input_ids, lambda: torch.arange(S, device=input_ids.device).unsqueeze(0)
                            .expand(B, S).contiguous())

    def _cached(self, kind: str, input_ids: torch.Tensor, make):
        """Per-shape constant id tensors (arange positions, zero token types), built once instead of every step."""
        key = (kind, tuple(input_ids.shape), input_ids.device)
        cache = self.__dict__.setdefault("_id_cache", {})
        t = cache.get(key)
        if t is None:
            if len(cache) > 16:
                cache.clear()
            t = cache[key] = make()
        return t

    def forward(self, input_ids, token_type_ids, rng: DropoutSeeds, training: bool,
                q8_for: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``q8_for``: the first encoder layer's QKV weight (fp8 path: the embedding kernel writes its fp8 operand)."""
        c = self.cfg
        pos = self.position_ids(input_ids)
        if token_type_ids is None and self.token_type_embeddings is not None:
            token_type_ids = self._cached("type0", input_ids, lambda: torch.zeros_like(input_ids))
        p = c.hidden_dropout_prob if training else 0.0
        return ops.embed_ln(input_ids, pos, token_type_ids, self.word_embeddings, self.position_embeddings,
                            self.token_type_embeddings, self.ln_weight, self.ln_bias, c.layer_norm_eps,
                            p, rng.next() if p else 0, pos_is_arange=c.model_type != "roberta", q8_for=q8_for)


class Encoder(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.cfg = cfg
        self.embeddings = Embeddings(cfg)
        self.layers = nn.ModuleList([EncoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])

    def forward(self, input_ids, attention_mask, token_type_ids, rng, training) -> torch.Tensor:
        B, S = input_ids.shape
        first_qkv = self.layers[0].qkv_weight if len(self.layers) else None
        h = self.embeddings(input_ids, token_type_ids, rng, training, q8_for=first_qkv).view(B * S, -1)
        mask_bias = ops.key_mask_bias(attention_mask) if attention_mask is not None else None
        n = len(self.layers)
        for i, layer in enumerate(self.layers):
            h = layer(h, mask_bias, B, S, rng, training, self.layers[i + 1].qkv_weight if i + 1 < n else None)
        return h.view(B, S, -1)


def _init_(module: nn.Module, cfg: ModelConfig, generator: Optional[torch.Generator] = None) -> None:
    """HF ``_init_weights``: N(0, initializer_range) for matrices/embeddings, zero bias, LN = (1, 0),
    zeroed padding rows ([dep: transformers/modeling_utils.py:2375-2420])."""
    std = cfg.initializer_range
    with torch.no_grad():
        for name, p in module.named_parameters():
            leaf = name.rsplit(".", 1)[-1]
            if any(t in ("ln", "ln1", "ln2") for t in leaf.split("_")):
                if leaf.endswith("weight"):
                    p.fill_(1.0)
                else:
                    p.zero_()
            elif leaf.endswith("bias"):
                p.zero_()
            else:
                p.normal_(0.0, std, generator=generator)
        emb = getattr(module, "encoder", None)
        if emb is not None:
            e = emb.embeddings
            if 0 <= cfg.pad_token_id < e.word_embeddings.shape[0]:
                e.word_embeddings[cfg.pad_token_id].zero_()
            if cfg.model_type == "roberta" and cfg.pad_token_id < e.position_embeddings.shape[0]:
                e.position_embeddings[cfg.pad_token_id].zero_()


class _Base(nn.Module):
    base_prefix = "bert"

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.cfg = cfg
        self.encoder = Encoder(cfg)
        self.rng = DropoutSeeds(0)

    # ----------------------------------------------------------------- HF name mapping
    def _embedding_hf_names(self) -> Iterator[Tuple[str, str, Optional[int], int]]:
        b = self.base_prefix
        yield f"{b}.embeddings.word_embeddings.weight", "encoder.embeddings.word_embeddings", None, 1
        yield f"{b}.embeddings.position_embeddings.weight", "encoder.embeddings.position_embeddings", None, 1
        if self.encoder.embeddings.token_type_embeddings is not None:
            yield f"{b}.embeddings.token_type_embeddings.weight", "encoder.embeddings.token_type_embeddings", None, 1
        yield f"{b}.embeddings.LayerNorm.weight", "encoder.embeddings.ln_weight", None, 1
        yield f"{b}.embeddings.LayerNorm.bias", "encoder.embeddings.ln_bias", None, 1

    def _layer_hf_names(self):
        distil = self.cfg.model_type == "distilbert"
        mid = "transformer" if distil else "encoder"
        for i in range(self.cfg.num_hidden_layers):
            yield from layer_hf_names(f"{self.base_prefix}.{mid}.layer.{i}.", f"encoder.layers.{i}.", distil)

    def _head_hf_names(self):
        return iter(())

    def hf_names(self) -> Iterator[Tuple[str, str, Optional[int], int]]:
        yield from self._embedding_hf_names()
        yield from self._layer_hf_names()
        yield from self._head_hf_names()

    def architecture(self) -> str:
        raise NotImplementedError

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters())


class TransformerForSequenceClassification(_Base):
    """BertForSequenceClassification / RobertaForSequenceClassification / DistilBertForSequenceClassification."""

    def __init__(self, cfg: ModelConfig):
        super().__init__(cfg)
        H, L = cfg.hidden_size, cfg.num_labels
        self.base_prefix = {"bert": "bert", "roberta": "roberta", "distilbert": "distilbert"}[cfg.model_type]
        if cfg.model_type == "bert":
            self.pooler_weight, self.pooler_bias = _param(H, H), _param(H)
        else:  # roberta classifier.dense / distilbert pre_classifier
            self.head_dense_weight, self.head_dense_bias = _param(H, H), _param(H)
        self.classifier_weight, self.classifier_bias = _param(L, H), _param(L)

    def architecture(self) -> str:
        return {"bert": "BertForSequenceClassification", "roberta": "RobertaForSequenceClassification",
                "distilbert": "DistilBertForSequenceClassification"}[self.cfg.model_type]

    def _head_hf_names(self):
        mt = self.cfg.model_type
        if mt == "bert":
            yield "bert.pooler.dense.weight", "pooler_weight", None, 1
            yield "bert.pooler.dense.bias", "pooler_bias", None, 1
            yield "classifier.weight", "classifier_weight", None, 1
            yield "classifier.bias", "classifier_bias", None, 1
        elif mt == "roberta":
            yield "classifier.dense.weight", "head_dense_weight", None, 1
            yield "classifier.dense.bias", "head_dense_bias", None, 1
            yield "classifier.out_proj.weight", "classifier_weight", None, 1
            yield "classifier.out_proj.bias", "classifier_bias", None, 1
        else:
            yield "pre_classifier.weight", "head_dense_weight", None, 1
            yield "pre_classifier.bias", "head_dense_bias", None, 1
            yield "classifier.weight", "classifier_weight", None, 1
            yield "classifier.bias", "classifier_bias", None, 1

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None):
        c = self.cfg
        training = self.training
        h = self.encoder(input_ids, attention_mask, token_type_ids, self.rng, training)
        # head on the [CLS] / <s> row (ops.cls_head: one fused kernel per direction after the dense GEMM on GPUs);
        # the dropout seeds are drawn in the same order as the unfused head always drew them
        if c.model_type == "bert":
            p = (c.classifier_dropout if c.classifier_dropout is not None else c.hidden_dropout_prob) if training else 0.0
            w1, b1, act, p_in, seed_in = self.pooler_weight, self.pooler_bias, "tanh", 0.0, 0
        elif c.model_type == "roberta":
            p = (c.classifier_dropout if c.classifier_dropout is not None else c.hidden_dropout_prob) if training else 0.0
            w1, b1, act, p_in = self.head_dense_weight, self.head_dense_bias, "tanh", p
            seed_in = self.rng.next() if p else 0
        else:
            p = c.seq_classif_dropout if training else 0.0
            w1, b1, act, p_in, seed_in = self.head_dense_weight, self.head_dense_bias, "relu", 0.0, 0
        seed = self.rng.next() if p else 0
        out = ops.cls_head(h, w1, b1, self.classifier_weight, self.classifier_bias, labels, act, p_in, seed_in, p, seed)
        if labels is not None:
            return out  # (loss, logits)
        return out


class RobertaForMaskedLM(_Base):
    """RoBERTa MLM (decoder tied to the word embeddings), for the roberta-large pretraining config."""

    base_prefix = "roberta"
    graph_safe = False  # the masked-token gather has a data-dependent size (no HIP-graph capture)

    # The decoder's vocabulary dimension (tied word embeddings, lm_head.bias) is padded to a multiple of this many
    # rows: 50265 -> 50432 for RoBERTa, so every GEMM of the head (logits forward, its dgrad and the tied-embedding
    # weight gradient) tiles on the hand-written MFMA kernels. The padding rows stay exactly zero (zero init, zero
    # gradient), the loss and the returned logits cover the real vocabulary only, and checkpoints keep HF's shapes
    # (models/hf_io.py slices on save, zero-pads on load).
    VOCAB_PAD = 256

    def __init__(self, cfg: ModelConfig):
        super().__init__(cfg)
        H = cfg.hidden_size
        self.vocab = cfg.vocab_size
        self.vocab_padded = -(-cfg.vocab_size // self.VOCAB_PAD) * self.VOCAB_PAD
        if self.vocab_padded != self.vocab:
            self.encoder.embeddings.word_embeddings = _param(self.vocab_padded, H)
        self.lm_dense_weight, self.lm_dense_bias = _param(H, H), _param(H)
        self.lm_ln_weight, self.lm_ln_bias = _param(H), _param(H)
        self.lm_bias = _param(self.vocab_padded)

    def padded_rows(self):
        """Internal parameter -> its HF row count (the rows beyond it are the zero vocabulary padding)."""
        return {"encoder.embeddings.word_embeddings": self.vocab, "lm_bias": self.vocab}

    @torch.no_grad()
    def zero_padding_rows(self) -> None:
        self.encoder.embeddings.word_embeddings[self.vocab:].zero_()
        self.lm_bias[self.vocab:].zero_()

    def architecture(self) -> str:
        return "RobertaForMaskedLM"

    def _head_hf_names(self):
        yield "lm_head.dense.weight", "lm_dense_weight", None, 1
        yield "lm_head.dense.bias", "lm_dense_bias", None, 1
        yield "lm_head.layer_norm.weight", "lm_ln_weight", None, 1
        yield "lm_head.layer_norm.bias", "lm_ln_bias", None, 1
        yield "lm_head.bias", "lm_bias", None, 1

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None):
        c = self.cfg
        h = self.encoder(input_ids, attention_mask, token_type_ids, self.rng, self.training)
        B, S, H = h.shape
        x = h.view(B * S, H)
        wemb = self.encoder.embeddings.word_embeddings
        if labels is not None:
            # only masked positions feed the (large-vocab) decoder: dense + GELU -> LN -> tied decoder -> CE
            loss, logits = ops.mlm_head(x, labels.view(-1), self.lm_dense_weight, self.lm_dense_bias, self.lm_ln_weight,
                                        self.lm_ln_bias, c.layer_norm_eps, wemb, self.lm_bias, self.vocab)
            return loss, logits
        x = ops.linear_gelu(x, self.lm_dense_weight, self.lm_dense_bias)
        x = ops.layer_norm(x, self.lm_ln_weight, self.lm_ln_bias, c.layer_norm_eps)
        logits = ops.linear(x, wemb[:self.vocab], self.lm_bias[:self.vocab])
        return logits.view(B, S, -1)


def build_model(cfg: ModelConfig, task: str = "sequence-classification", seed: Optional[int] = 0) -> _Base:
    if task in ("sequence-classification", "seq-cls"):
        m = TransformerForSequenceClassification(cfg)
    elif task in ("masked-lm", "mlm"):
        if cfg.model_type != "roberta":
            raise ValueError("masked-lm is provided for roberta configs")
        m = RobertaForMaskedLM(cfg)
    else:
        raise ValueError(task)
    g = None
    if seed is not None:
        g = torch.Generator()
        g.manual_seed(int(seed))
    _init_(m, cfg, g)
    if hasattr(m, "zero_padding_rows"):
        m.zero_padding_rows()
    return m
