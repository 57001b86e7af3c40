"""Offline tokenizers.

The reference loads ``AutoTokenizer.from_pretrained(model_name_or_path)`` from the HF hub
(``scripts/train.py:69``) — a Rust ``tokenizers`` fast tokenizer. There is no hub here, so:

* a local model directory with ``tokenizer.json`` is loaded with the ``tokenizers`` library
  (same Rust backend as the reference);
* otherwise a WordPiece tokenizer is built from a generated vocabulary (BERT special tokens at
  their standard ids: [PAD]=0, [UNK]=100, [CLS]=101, [SEP]=102, [MASK]=103) so the text path and
  ``tokenizer.save_pretrained`` (``scripts/train.py:183``) still work offline.
"""
from __future__ import annotations

import json
import os
import string
from typing import Dict, List, Optional, Sequence

import numpy as np

SPECIAL_BERT = {"[PAD]": 0, "[UNK]": 100, "[CLS]": 101, "[SEP]": 102, "[MASK]": 103}


def _generated_vocab(vocab_size: int) -> List[str]:
    vocab = [f"[unused{i}]" for i in range(vocab_size)]
    for tok, i in SPECIAL_BERT.items():
        if i < vocab_size:
            vocab[i] = tok
    pieces = list(string.ascii_lowercase) + list(string.digits) + list(string.punctuation)
    pieces += ["##" + c for c in string.ascii_lowercase + string.digits]
    common = ("the a an and or but if of to in on at for with is was are were be been this that it its i you he "
              "she they we movie film good bad great terrible awful best worst love hate not no very really story "
              "acting plot character characters one two time just like even would could see watch watched "
              "funny boring excellent wonderful poor waste").split()
    pieces += common
    seen = set()
    pieces = [x for x in pieces if not (x in seen or seen.add(x))]
    nxt = 104
    for p in pieces:
        while nxt < vocab_size and vocab[nxt] in SPECIAL_BERT:
            nxt += 1
        if nxt >= vocab_size:
            break
        vocab[nxt] = p
        nxt += 1
    return vocab


class Tokenizer:
    """Thin wrapper over a ``tokenizers.Tokenizer`` with the HF call convention we need."""

    def __init__(self, backend, model_max_length: int = 512, pad_token_id: int = 0, name: str = ""):
        self.backend = backend
        self.model_max_length = int(model_max_length)
        self.pad_token_id = int(pad_token_id)
        self.name = name

    @classmethod
    def generated_wordpiece(cls, vocab_size: int = 30522, model_max_length: int = 512) -> "Tokenizer":
        from tokenizers import Tokenizer as TK
        from tokenizers import decoders, models, normalizers, pre_tokenizers, processors

        vocab = {t: i for i, t in enumerate(_generated_vocab(vocab_size))}
        tk = TK(models.WordPiece(vocab=vocab, unk_token="[UNK]", max_input_chars_per_word=100))
        tk.normalizer = normalizers.BertNormalizer(lowercase=True)
        tk.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
        tk.post_processor = processors.TemplateProcessing(
            single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
            special_tokens=[("[CLS]", 101), ("[SEP]", 102)])
        tk.decoder = decoders.WordPiece()
        return cls(tk, model_max_length, 0, "generated-wordpiece")

    @classmethod
    def from_dir(cls, path: str, model_max_length: int = 512) -> Optional["Tokenizer"]:
        f = os.path.join(path, "tokenizer.json")
        if not os.path.isfile(f):
            return None
        from tokenizers import Tokenizer as TK

        tk = TK.from_file(f)
        pad = 0
        cfgf = os.path.join(path, "tokenizer_config.json")
        if os.path.isfile(cfgf):
            with open(cfgf) as fh:
                c = json.load(fh)
            model_max_length = int(min(c.get("model_max_length", model_max_length), 1 << 20))
            pt = c.get("pad_token")
            if isinstance(pt, str) and tk.token_to_id(pt) is not None:
                pad = tk.token_to_id(pt)
        return cls(tk, model_max_length, pad, path)

    def encode_batch(self, texts: Sequence[str], max_length: int) -> Dict[str, np.ndarray]:
        """truncation=True + pad to ``max_length`` (the reference's effective padding)."""
        self.backend.enable_truncation(max_length)
        self.backend.enable_padding(length=max_length, pad_id=self.pad_token_id)
        enc = self.backend.encode_batch(list(texts))
        ids = np.asarray([e.ids for e in enc], dtype=np.int32)
        mask = np.asarray([e.attention_mask for e in enc], dtype=np.int8)
        return {"input_ids": ids, "attention_mask": mask}

    def save_pretrained(self, save_directory: str) -> List[str]:
        os.makedirs(save_directory, exist_ok=True)
        tj = os.path.join(save_directory, "tokenizer.json")
        self.backend.save(tj)
        cfg = {"model_max_length": self.model_max_length, "do_lower_case": True, "pad_token": "[PAD]",
               "unk_token": "[UNK]", "cls_token": "[CLS]", "sep_token": "[SEP]", "mask_token": "[MASK]",
               "tokenizer_class": "BertTokenizerFast"}
        tc = os.path.join(save_directory, "tokenizer_config.json")
        with open(tc, "w") as f:
            json.dump(cfg, f, indent=2)
        sm = os.path.join(save_directory, "special_tokens_map.json")
        with open(sm, "w") as f:
            json.dump({k: cfg[k] for k in ("pad_token", "unk_token", "cls_token", "sep_token", "mask_token")}, f,
                      indent=2)
        return [tj, tc, sm]


def load_tokenizer(model_name_or_path: Optional[str], vocab_size: int, model_max_length: int = 512) -> Tokenizer:
    if model_name_or_path and os.path.isdir(model_name_or_path):
        t = Tokenizer.from_dir(model_name_or_path, model_max_length)
        if t is not None:
            return t
    return Tokenizer.generated_wordpiece(vocab_size, model_max_length)
