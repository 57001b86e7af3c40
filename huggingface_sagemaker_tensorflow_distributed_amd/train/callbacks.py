"""Callbacks and checkpoint/resume.

* :class:`ModelCheckpoint` — the rank-0 ``ModelCheckpoint("./checkpoint-{epoch}.h5")`` that the
  reference ships commented out (``scripts/train.py:135-137``), enabled by ``--save_every_epoch``;
  writes ``checkpoint-{epoch}/`` in HF layout + optimizer state + trainer state.
* :func:`load_checkpoint` — the restore path the broadcast-callback comment mentions
  (``scripts/train.py:132``) but the reference never implements (``--resume_from``).
"""
from __future__ import annotations

import json
import logging
import os
import random
import time

import numpy as np
import torch

from ..models.hf_io import hf_state_dict, load_hf_state_dict, read_checkpoint, save_pretrained
from ..parallel import backend

logger = logging.getLogger(__name__)


class Callback:
    def on_train_begin(self, trainer):
        pass

    def on_batch_end(self, trainer, step):
        pass

    def on_epoch_end(self, trainer, epoch, logs):
        pass

    def on_train_end(self, trainer):
        pass


def master_state_dict(model, store):
    """HF-layout fp32 weights taken from the fp32 master copy (not the bf16 compute copy)."""
    saved = []
    for seg, p in zip(store.segments, store.params):
        saved.append(p.data)
        p.data = store.master[seg.offset:seg.offset + seg.numel].view(seg.shape)
    try:
        return hf_state_dict(model)
    finally:
        for p, d in zip(store.params, saved):
            p.data = d


def save_checkpoint(path: str, trainer, epoch: int) -> None:
    if backend.rank() == 0:
        os.makedirs(path, exist_ok=True)
        save_pretrained(trainer.model, path, state_dict=master_state_dict(trainer.model, trainer.store))
        torch.save(trainer.optimizer.state_dict(), os.path.join(path, "optimizer.pt"))
        with open(os.path.join(path, "trainer_state.json"), "w") as f:
            json.dump({"epoch": epoch, "global_step": trainer.global_step,
                       "python_rng": random.getstate()[1][0], "numpy_seed": int(np.random.get_state()[1][0])}, f)
        logger.info("checkpoint written to %s", path)
    backend.barrier()


def load_checkpoint(path: str, trainer) -> dict:
    """Restore weights, optimizer and step; returns the trainer state (``epoch`` = epochs completed, the
    ``initial_epoch`` a resumed ``fit`` starts from)."""
    sd = read_checkpoint(path)
    if sd is None:
        raise FileNotFoundError(path)
    store = trainer.store
    # load into master through temporary views
    saved = []
    for seg, p in zip(store.segments, store.params):
        saved.append(p.data)
        p.data = store.master[seg.offset:seg.offset + seg.numel].view(seg.shape)
    try:
        load_hf_state_dict(trainer.model, sd)
    finally:
        for p, d in zip(store.params, saved):
            p.data = d
    store.sync_compute_from_master()
    opt = os.path.join(path, "optimizer.pt")
    if os.path.isfile(opt):
        trainer.optimizer.load_state_dict(torch.load(opt, map_location="cpu", weights_only=True))
    st = {}
    sf = os.path.join(path, "trainer_state.json")
    if os.path.isfile(sf):
        with open(sf) as f:
            st = json.load(f)
        trainer.global_step = int(st.get("global_step", 0))
    st.setdefault("epoch", 0)
    return st


class ModelCheckpoint(Callback):
    def __init__(self, pattern: str = "checkpoint-{epoch}"):
        self.pattern = pattern

    def on_epoch_end(self, trainer, epoch, logs):
        save_checkpoint(self.pattern.format(epoch=epoch + 1), trainer, epoch + 1)


class FaultInjection(Callback):
    """Test hook: ``HSD_FAULT_RANK`` / ``HSD_FAULT_STEP`` crash one rank mid-training;
    with ``HSD_FAULT_HANG=1`` that rank hangs inside its next step instead (a stand-in for a stuck kernel or
    collective), which only the step watchdog (``--step_watchdog``) can turn into a failed job."""

    def __init__(self):
        self.rank = int(os.environ.get("HSD_FAULT_RANK", "-1"))
        self.step = int(os.environ.get("HSD_FAULT_STEP", "-1"))
        self.hang = os.environ.get("HSD_FAULT_HANG", "0") == "1"

    def on_train_begin(self, trainer):
        if self.hang and backend.rank() == self.rank and self.step >= 0:
            inner = trainer._forward_loss

            def hanging_forward(batch):
                if trainer.global_step >= self.step:
                    while True:  # never returns: the watchdog ends the process
                        time.sleep(3600)
                return inner(batch)

            trainer._forward_loss = hanging_forward

    def on_batch_end(self, trainer, step):
        if not self.hang and backend.rank() == self.rank and trainer.global_step >= self.step >= 0:
            raise SystemExit(f"injected fault on rank {self.rank} at step {trainer.global_step}")


class BroadcastGlobalVariablesCallback(Callback):
    """``hvd.callbacks.BroadcastGlobalVariablesCallback(root_rank)`` (``scripts/train.py:133``): every rank starts
    from ``root_rank``'s weights (and optimizer state). Horovod's Keras callback broadcasts at the end of the first
    batch, after the optimizer slots exist; here the flat master / moment buffers exist from construction, so the
    broadcast happens BEFORE step 1 and the first update is already identical on every rank."""

    def __init__(self, root_rank: int = 0):
        self.root_rank = int(root_rank)

    def on_train_begin(self, trainer):
        from ..parallel.collectives import broadcast_parameters

        if backend.is_distributed():
            broadcast_parameters(trainer.store, trainer.optimizer, src=self.root_rank)


class MetricAverageCallback(Callback):
    """``hvd.callbacks.MetricAverageCallback()``: the epoch metrics the Trainer reports are already exact global
    averages (an all-reduce of loss-sum / correct / count), so this exists for source
    compatibility and does nothing."""
