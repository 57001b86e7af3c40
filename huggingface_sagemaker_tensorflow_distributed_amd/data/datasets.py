"""Datasets: synthetic (default, no network) and local IMDB / SST-2 text.

Reference data path (``scripts/train.py:71-100``): ``load_dataset("imdb")``, tokenize with
``truncation=True``, pad every example to exactly ``tokenizer.model_max_length`` (512), keep
``input_ids``/``attention_mask``/``label`` — ``token_type_ids`` are never fed.

Offline here, so:

* ``synthetic``: a learnable binary task of the same tensor shapes. Label 1 sequences contain a
  "positive" marker token at a random position, label 0 sequences a "negative" one; real-length
  variation comes from a padded tail (or full length for throughput runs, which matches IMDB at
  S=128: almost every review is longer than 128 tokens and is truncated to full length).
* ``imdb`` / ``sst2`` / a path: read from a local directory (HF ``save_to_disk`` dir, parquet,
  csv/tsv, jsonl, or the raw ``aclImdb/{train,test}/{pos,neg}/*.txt`` tree).
"""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

POS_MARK = 2204  # "good" in bert-base-uncased's vocab
NEG_MARK = 2919  # "bad"


@dataclass
class ArrayDataset:
    input_ids: np.ndarray        # [N, S] int32
    attention_mask: np.ndarray   # [N, S] int8
    labels: np.ndarray           # [N] int64 (or [N, S] for MLM)

    def __len__(self) -> int:
        return int(self.input_ids.shape[0])

    @property
    def seq_len(self) -> int:
        return int(self.input_ids.shape[1])


def synthetic_classification(num_examples: int, seq_len: int, vocab_size: int, seed: int = 0,
                             full_length: bool = False, num_labels: int = 2, cls_id: int = 101, sep_id: int = 102,
                             pad_id: int = 0) -> ArrayDataset:
    rng = np.random.default_rng(seed)
    lo = 1000 if vocab_size > 4000 else 4
    ids = rng.integers(lo, vocab_size, size=(num_examples, seq_len), dtype=np.int64)
    labels = rng.integers(0, num_labels, size=(num_examples,), dtype=np.int64)
    if full_length:
        lengths = np.full(num_examples, seq_len)
    else:
        lengths = rng.integers(max(4, seq_len // 4), seq_len + 1, size=num_examples)
    marks = np.array([POS_MARK, NEG_MARK] + [NEG_MARK + 1 + i for i in range(num_labels - 2)]) % vocab_size
    for i in range(num_examples):
        L = int(lengths[i])
        ids[i, 0] = cls_id % vocab_size
        ids[i, L - 1] = sep_id % vocab_size
        pos = int(rng.integers(1, max(2, L - 1)))
        ids[i, pos] = marks[labels[i]]
        ids[i, L:] = pad_id
    mask = (np.arange(seq_len)[None, :] < lengths[:, None]).astype(np.int8)
    return ArrayDataset(ids.astype(np.int32), mask, labels)


def synthetic_mlm(num_examples: int, seq_len: int, vocab_size: int, seed: int = 0, mask_id: int = 50264,
                  mlm_probability: float = 0.15, bos_id: int = 0, eos_id: int = 2) -> ArrayDataset:
    rng = np.random.default_rng(seed)
    ids = rng.integers(3, vocab_size, size=(num_examples, seq_len), dtype=np.int64)
    ids[:, 0] = bos_id
    ids[:, -1] = eos_id
    labels = np.full_like(ids, -100)
    sel = rng.random(ids.shape) < mlm_probability
    sel[:, 0] = sel[:, -1] = False
    labels[sel] = ids[sel]
    ids[sel] = mask_id % vocab_size
    return ArrayDataset(ids.astype(np.int32), np.ones_like(ids, dtype=np.int8), labels)


# ------------------------------------------------------------------------------------------ text
def _read_table(path: str) -> Tuple[List[str], List[int]]:
    ext = os.path.splitext(path)[1].lower()
    if ext == ".parquet":
        import pyarrow.parquet as pq

        t = pq.read_table(path).to_pydict()
    elif ext in (".jsonl", ".json"):
        rows = [json.loads(l) for l in open(path) if l.strip()]
        t = {k: [r[k] for r in rows] for k in rows[0]}
    elif ext in (".csv", ".tsv"):
        import pandas as pd

        t = pd.read_csv(path, sep="\t" if ext == ".tsv" else ",").to_dict(orient="list")
    else:
        raise ValueError(f"unsupported dataset file {path}")
    text_key = "text" if "text" in t else "sentence"
    return [str(x) for x in t[text_key]], [int(x) for x in t["label"]]


def load_text_split(name_or_path: str, split: str, dataset_dir: Optional[str] = None) -> Tuple[List[str], List[int]]:
    """``split`` in {"train", "test"}; SST-2's ``validation`` serves as its test split."""
    roots = [p for p in (name_or_path, dataset_dir, os.path.join(dataset_dir or "", name_or_path)) if p]
    for root in roots:
        if not os.path.exists(root):
            continue
        if os.path.isfile(root):
            return _read_table(root)
        # HF datasets save_to_disk
        if os.path.isfile(os.path.join(root, "dataset_dict.json")):
            from datasets import load_from_disk

            dd = load_from_disk(root)
            sp = split if split in dd else ("validation" if split == "test" and "validation" in dd else split)
            d = dd[sp]
            key = "text" if "text" in d.column_names else "sentence"
            return list(d[key]), list(d["label"])
        cands = []
        for sp in ([split] if split == "train" else [split, "validation", "dev"]):
            cands += sorted(glob.glob(os.path.join(root, f"{sp}*.parquet")))
            cands += sorted(glob.glob(os.path.join(root, "*", f"{sp}*.parquet")))
            for ext in ("jsonl", "csv", "tsv"):
                cands += sorted(glob.glob(os.path.join(root, f"{sp}*.{ext}")))
        if cands:
            texts, labels = [], []
            for c in cands:
                t, l = _read_table(c)
                texts += t
                labels += l
            return texts, labels
        raw = os.path.join(root, split)
        if os.path.isdir(os.path.join(raw, "pos")):  # aclImdb layout
            texts, labels = [], []
            for lab, sub in ((0, "neg"), (1, "pos")):
                for f in sorted(glob.glob(os.path.join(raw, sub, "*.txt"))):
                    texts.append(open(f, encoding="utf-8").read())
                    labels.append(lab)
            return texts, labels
    raise FileNotFoundError(f"dataset {name_or_path!r} split {split!r} not found locally "
                            f"(no network: pass --dataset_dir or use --dataset synthetic)")


def tokenize_dataset(tokenizer, texts: List[str], labels: List[int], max_length: int,
                     chunk: int = 1000) -> ArrayDataset:
    ids, mask = [], []
    for i in range(0, len(texts), chunk):  # the reference maps in 1000-row batches
        enc = tokenizer.encode_batch(texts[i:i + chunk], max_length)
        ids.append(enc["input_ids"])
        mask.append(enc["attention_mask"])
    return ArrayDataset(np.concatenate(ids), np.concatenate(mask), np.asarray(labels, dtype=np.int64))
