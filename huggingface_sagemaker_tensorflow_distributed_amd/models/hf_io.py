"""HF-compatible checkpoint I/O (``save_pretrained`` / ``from_pretrained``).

The reference calls ``model.save_pretrained(args.model_dir)`` (``scripts/train.py:182``), which in
TF writes ``tf_model.h5`` + ``config.json``. We write the HF PyTorch layout, ``config.json`` +
``model.safetensors`` with HF key names, so
``transformers.AutoModelForSequenceClassification.from_pretrained(model_dir)`` loads it unchanged.
"""
from __future__ import annotations

import json
import logging
import os
from typing import Dict, Optional

import torch

from .bert import _Base, build_model
from .config import ModelConfig, resolve_config

logger = logging.getLogger(__name__)

WEIGHTS_NAME = "model.safetensors"
CONFIG_NAME = "config.json"


def hf_state_dict(model: _Base, dtype: Optional[torch.dtype] = torch.float32) -> Dict[str, torch.Tensor]:
    """Internal (fused) parameters -> HF-named tensors (Q/K/V split back apart)."""
    params = dict(model.named_parameters())
    padded = model.padded_rows() if hasattr(model, "padded_rows") else {}
    out: Dict[str, torch.Tensor] = {}
    for hf_key, ikey, split, nsplit in model.hf_names():
        t = params[ikey].detach()
        if ikey in padded:
            t = t[:padded[ikey]]  # drop the zero vocabulary padding rows
        if split is not None:
            t = t.chunk(nsplit, dim=0)[split]
        t = t.to("cpu")
        if dtype is not None:
            t = t.to(dtype)
        out[hf_key] = t.contiguous().clone()
    return out


def load_hf_state_dict(model: _Base, sd: Dict[str, torch.Tensor], strict: bool = False) -> Dict[str, list]:
    """HF-named tensors -> internal parameters. Missing head weights keep their fresh init (like HF)."""
    params = dict(model.named_parameters())
    base = model.base_prefix + "."
    missing, used = [], set()
    # a bare BaseModel checkpoint has no "bert." prefix: accept both
    def lookup(k):
        if k in sd:
            return k
        if k.startswith(base) and k[len(base):] in sd:
            return k[len(base):]
        return None

    padded = model.padded_rows() if hasattr(model, "padded_rows") else {}
    pending: Dict[str, list] = {}
    for hf_key, ikey, split, nsplit in model.hf_names():
        k = lookup(hf_key)
        if k is None:
            missing.append(hf_key)
            continue
        used.add(k)
        pending.setdefault(ikey, [None] * nsplit)[split or 0] = sd[k]
    with torch.no_grad():
        for ikey, parts in pending.items():
            if any(x is None for x in parts):
                missing.append(ikey)
                continue
            t = parts[0] if len(parts) == 1 else torch.cat(parts, dim=0)
            dst = params[ikey]
            if ikey in padded and t.shape[0] == padded[ikey] and tuple(t.shape[1:]) == tuple(dst.shape[1:]):
                dst.zero_()  # HF rows, then the zero vocabulary padding
                dst[:t.shape[0]].copy_(t.to(dst.dtype))
                continue
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"shape mismatch for {ikey}: checkpoint {tuple(t.shape)} vs model {tuple(dst.shape)}")
            dst.copy_(t.to(dst.dtype))
    unexpected = [k for k in sd if k not in used]
    if strict and (missing or unexpected):
        raise KeyError(f"missing={missing} unexpected={unexpected}")
    return {"missing": missing, "unexpected": unexpected}


def save_pretrained(model: _Base, save_directory: str, weights_dtype: torch.dtype = torch.float32,
                    state_dict: Optional[Dict[str, torch.Tensor]] = None) -> None:
    from safetensors.torch import save_file

    os.makedirs(save_directory, exist_ok=True)
    cfg_dict = model.cfg.to_hf_dict(model.architecture())
    with open(os.path.join(save_directory, CONFIG_NAME), "w") as f:
        json.dump(cfg_dict, f, indent=2, sort_keys=True)
    sd = state_dict if state_dict is not None else hf_state_dict(model, weights_dtype)
    save_file(sd, os.path.join(save_directory, WEIGHTS_NAME), metadata={"format": "pt"})
    logger.info("Model weights saved in %s", os.path.join(save_directory, WEIGHTS_NAME))


def read_checkpoint(path: str) -> Optional[Dict[str, torch.Tensor]]:
    """Load weights with loaders that execute nothing from the file."""
    st = os.path.join(path, WEIGHTS_NAME)
    if os.path.isfile(st):
        from safetensors.torch import load_file

        return load_file(st)
    pt = os.path.join(path, "pytorch_model.bin")
    if os.path.isfile(pt):
        return torch.load(pt, map_location="cpu", weights_only=True)
    return None


def from_pretrained(name_or_path: str, task: str = "sequence-classification", num_labels: Optional[int] = None,
                    seed: Optional[int] = 0) -> _Base:
    cfg = resolve_config(name_or_path, num_labels=num_labels)
    model = build_model(cfg, task=task, seed=seed)
    model.weights_source = "random-init"  # what the run's provenance record reports
    if os.path.isdir(name_or_path):
        sd = read_checkpoint(name_or_path)
        if sd is not None:
            info = load_hf_state_dict(model, sd)
            model.weights_source = os.path.abspath(name_or_path)
            if info["missing"]:
                logger.info("Some weights were newly initialized: %s", info["missing"])
        else:
            logger.warning("%s has no weights file; using random init", name_or_path)
    else:
        logger.info("offline registry config %r: random-init weights (no hub access)", name_or_path)
    return model
