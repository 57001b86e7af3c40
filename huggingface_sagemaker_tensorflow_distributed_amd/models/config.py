"""Model configuration + offline registry.

The reference resolves ``--model_name_or_path`` against the HF hub
(``TFAutoModelForSequenceClassification.from_pretrained``, ``scripts/train.py:117``). There is no
network here, so known hub ids map to built-in configs (values from the public model cards /
[dep: transformers/models/*/configuration_*.py] defaults), and any local directory holding a
``config.json`` works too (SURVEY.md §2.7 ``--model_name_or_path``).
"""
from __future__ import annotations

import copy
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class ModelConfig:
    model_type: str = "bert"  # bert | roberta | distilbert
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    classifier_dropout: Optional[float] = None
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0
    bos_token_id: Optional[int] = None
    eos_token_id: Optional[int] = None
    num_labels: int = 2
    tie_word_embeddings: bool = True
    # distilbert-only
    sinusoidal_pos_embds: bool = False
    seq_classif_dropout: float = 0.2
    # bookkeeping
    name_or_path: str = ""
    model_max_length: int = 512
    id2label: Optional[Dict[str, str]] = None
    extra: Dict[str, Any] = field(default_factory=dict)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(copy.deepcopy(self), **kw)

    # ---- HF config.json round trip -------------------------------------------------------
    def to_hf_dict(self, architecture: Optional[str] = None) -> Dict[str, Any]:
        mt = self.model_type
        labels = self.id2label or {str(i): f"LABEL_{i}" for i in range(self.num_labels)}
        common = {
            "model_type": mt,
            "vocab_size": self.vocab_size,
            "initializer_range": self.initializer_range,
            "pad_token_id": self.pad_token_id,
            "id2label": labels,
            "label2id": {v: int(k) for k, v in labels.items()},
            "torch_dtype": "float32",
        }
        if architecture:
            common["architectures"] = [architecture]
        if mt == "distilbert":
            common.update({
                "dim": self.hidden_size, "n_layers": self.num_hidden_layers,
                "n_heads": self.num_attention_heads, "hidden_dim": self.intermediate_size,
                "activation": self.hidden_act, "dropout": self.hidden_dropout_prob,
                "attention_dropout": self.attention_probs_dropout_prob,
                "max_position_embeddings": self.max_position_embeddings,
                "sinusoidal_pos_embds": self.sinusoidal_pos_embds,
                "seq_classif_dropout": self.seq_classif_dropout,
                "qa_dropout": 0.1, "tie_weights_": True,
            })
        else:
            common.update({
                "hidden_size": self.hidden_size, "num_hidden_layers": self.num_hidden_layers,
                "num_attention_heads": self.num_attention_heads,
                "intermediate_size": self.intermediate_size, "hidden_act": self.hidden_act,
                "hidden_dropout_prob": self.hidden_dropout_prob,
                "attention_probs_dropout_prob": self.attention_probs_dropout_prob,
                "max_position_embeddings": self.max_position_embeddings,
                "type_vocab_size": self.type_vocab_size, "layer_norm_eps": self.layer_norm_eps,
                "classifier_dropout": self.classifier_dropout,
                "position_embedding_type": "absolute", "use_cache": True,
            })
            if self.bos_token_id is not None:
                common["bos_token_id"] = self.bos_token_id
            if self.eos_token_id is not None:
                common["eos_token_id"] = self.eos_token_id
        return common

    @classmethod
    def from_hf_dict(cls, d: Dict[str, Any]) -> "ModelConfig":
        mt = d.get("model_type", "bert")
        labels = d.get("id2label")
        nl = len(labels) if labels else d.get("num_labels", 2)
        if mt == "distilbert":
            return cls(
                model_type="distilbert", vocab_size=d.get("vocab_size", 30522),
                hidden_size=d.get("dim", 768), num_hidden_layers=d.get("n_layers", 6),
                num_attention_heads=d.get("n_heads", 12), intermediate_size=d.get("hidden_dim", 3072),
                hidden_act=d.get("activation", "gelu"), hidden_dropout_prob=d.get("dropout", 0.1),
                attention_probs_dropout_prob=d.get("attention_dropout", 0.1),
                max_position_embeddings=d.get("max_position_embeddings", 512), type_vocab_size=0,
                initializer_range=d.get("initializer_range", 0.02), layer_norm_eps=1e-12,
                pad_token_id=d.get("pad_token_id", 0), num_labels=nl,
                sinusoidal_pos_embds=d.get("sinusoidal_pos_embds", False),
                seq_classif_dropout=d.get("seq_classif_dropout", 0.2), id2label=labels,
            )
        return cls(
            model_type=mt, vocab_size=d.get("vocab_size", 30522), hidden_size=d.get("hidden_size", 768),
            num_hidden_layers=d.get("num_hidden_layers", 12),
            num_attention_heads=d.get("num_attention_heads", 12),
            intermediate_size=d.get("intermediate_size", 3072), hidden_act=d.get("hidden_act", "gelu"),
            hidden_dropout_prob=d.get("hidden_dropout_prob", 0.1),
            attention_probs_dropout_prob=d.get("attention_probs_dropout_prob", 0.1),
            classifier_dropout=d.get("classifier_dropout"),
            max_position_embeddings=d.get("max_position_embeddings", 512),
            type_vocab_size=d.get("type_vocab_size", 2), initializer_range=d.get("initializer_range", 0.02),
            layer_norm_eps=d.get("layer_norm_eps", 1e-12), pad_token_id=d.get("pad_token_id", 0),
            bos_token_id=d.get("bos_token_id"), eos_token_id=d.get("eos_token_id"),
            num_labels=nl, id2label=labels,
        )


_BERT_BASE = ModelConfig()
_BERT_LARGE = ModelConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)
_DISTILBERT = ModelConfig(model_type="distilbert", num_hidden_layers=6, type_vocab_size=0, seq_classif_dropout=0.2)
_ROBERTA_BASE = ModelConfig(model_type="roberta", vocab_size=50265, max_position_embeddings=514, type_vocab_size=1,
                            layer_norm_eps=1e-5, pad_token_id=1, bos_token_id=0, eos_token_id=2)
_ROBERTA_LARGE = _ROBERTA_BASE.replace(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                                       intermediate_size=4096)

REGISTRY: Dict[str, ModelConfig] = {
    "bert-base-uncased": _BERT_BASE,
    "bert-base-cased": _BERT_BASE.replace(vocab_size=28996),
    "bert-large-uncased": _BERT_LARGE,
    "bert-large-uncased-whole-word-masking": _BERT_LARGE,
    "bert-large-cased": _BERT_LARGE.replace(vocab_size=28996),
    "distilbert-base-uncased": _DISTILBERT,
    "roberta-base": _ROBERTA_BASE,
    "roberta-large": _ROBERTA_LARGE,
    # tiny configs for tests / plumbing
    "hsd-tiny-bert": ModelConfig(vocab_size=1024, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                 intermediate_size=128, max_position_embeddings=128),
    "hsd-tiny-distilbert": ModelConfig(model_type="distilbert", vocab_size=1024, hidden_size=64,
                                       num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                                       max_position_embeddings=128, type_vocab_size=0),
    "hsd-tiny-roberta": ModelConfig(model_type="roberta", vocab_size=1024, hidden_size=64, num_hidden_layers=2,
                                    num_attention_heads=4, intermediate_size=128, max_position_embeddings=130,
                                    type_vocab_size=1, layer_norm_eps=1e-5, pad_token_id=1, bos_token_id=0,
                                    eos_token_id=2),
}
for _k in ("distilbert-base-uncased-finetuned-sst-2-english",):
    REGISTRY[_k] = _DISTILBERT


def resolve_config(name_or_path: Optional[str], num_labels: Optional[int] = None) -> ModelConfig:
    if not name_or_path:
        name_or_path = "bert-base-uncased"
    if os.path.isdir(name_or_path):
        with open(os.path.join(name_or_path, "config.json")) as f:
            cfg = ModelConfig.from_hf_dict(json.load(f))
    else:
        key = name_or_path.split("/")[-1] if name_or_path not in REGISTRY else name_or_path
        if key not in REGISTRY:
            raise KeyError(f"unknown model {name_or_path!r}: not a local directory and not in the offline "
                           f"registry {sorted(REGISTRY)}")
        cfg = copy.deepcopy(REGISTRY[key])
    cfg.name_or_path = name_or_path
    if num_labels is not None and num_labels != cfg.num_labels:
        cfg.num_labels = num_labels
        cfg.id2label = None
    return cfg
