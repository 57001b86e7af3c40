"""Keras-equivalent ``fit`` / ``evaluate`` loop (reference L6: ``model.compile/fit/evaluate``,
``scripts/train.py:123,145,170``).

One training step (SURVEY.md §3.3 'Our step'):

1. new dropout seeds for the step, gradient buffer zeroed (one memset of the flat buffer);
2. forward through the fused HIP kernels, ``SparseCategoricalCrossentropy(from_logits)`` mean loss;
3. backward: kernels write parameter gradients straight into the flat ``main_grad`` buffer and each
   completed bucket starts its RCCL all-reduce while backward continues;
4. wait for the buckets, one fused-Adam launch (``1/N`` folded in) that also refreshes the bf16
   weights.

Metrics stay on the device (no host sync per step) and are all-reduced at epoch end so the
reported history is global.
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional

import torch

from .. import ops
from ..obs.profiler import range as prange
from ..parallel import backend
from ..optim.adam import FusedAdam
from ..parallel.collectives import allreduce_sums, params_in_sync

logger = logging.getLogger(__name__)


@dataclass
class History:
    history: Dict[str, List[float]] = field(default_factory=dict)
    epoch: List[int] = field(default_factory=list)

    def append(self, epoch: int, logs: Dict[str, float]) -> None:
        self.epoch.append(epoch)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(v)

    def __repr__(self) -> str:  # mirrors the keras object repr that the reference logs
        return f"<History epochs={len(self.epoch)} keys={list(self.history)}>"


class _Meter:
    """Device-side running sums: loss·n, correct, n."""

    def __init__(self, device):
        self.t = torch.zeros(3, dtype=torch.float64, device=device)
        self._pending: List[torch.Tensor] = []

    def _fold(self) -> None:
        if self._pending:
            s = torch.stack(self._pending).double().sum(0)
            self.t += s[[3, 1, 2]]
            self._pending.clear()

    def update(self, loss: torch.Tensor, logits: torch.Tensor, labels: torch.Tensor, static: bool = False) -> None:
        """``static``: ``loss`` / ``logits`` are a captured graph's output buffers, overwritten by the next replay."""
        fused_stats = getattr(loss, "_hsd_stats", None)
        if fused_stats is not None:
            if static:
                fused_stats = fused_stats.clone()
            # the fused head already counted {loss sum, hits, rows} on the device: keep the tensor, add them up
            # when the metrics are read (no kernels per step)
            self._pending.append(fused_stats)
            if len(self._pending) >= 256:
                self._fold()
            return
        # classification: one label per logits row, -100 on the rows that only pad the eval shards;
        # MLM: logits only for the non-ignored (masked) tokens. Either way n counts the scored rows.
        n = labels.ne(-100).sum()
        fused = getattr(loss, "_hsd_correct", None)
        if fused is not None:
            correct = fused
        elif logits.dim() == 2 and logits.shape[0] == labels.numel():
            correct = ops.accuracy_count(logits, labels)
        else:
            correct = torch.zeros((), device=logits.device)
        nd = n.to(self.t.device).double()
        # an all-padding batch has a NaN mean loss on the torch path: it contributes nothing
        lsum = torch.where(nd > 0, loss.detach().double() * nd, torch.zeros_like(nd))
        upd = torch.stack([lsum, correct.to(self.t.device).double(), nd])
        self.t += upd

    def result(self, global_: bool = True) -> Dict[str, float]:
        self._fold()
        vals = self.t.tolist()
        if global_:
            vals = allreduce_sums(vals, self.t.device)
        loss_sum, correct, n = vals
        n = max(n, 1.0)
        return {"loss": loss_sum / n, "sparse_categorical_accuracy": correct / n}


class Trainer:
    # eager GPU steps: the fused Adam clears each gradient slice it consumes, replacing the memset ahead of the next
    # step's forward (False: a separate zero_grad every step)
    zero_grad_in_optimizer = True

    def __init__(self, model, store, optimizer, bucketer=None, device=None, grad_accum: int = 1,
                 check_sync: int = 0, log_every: int = 50, step_watchdog: float = 0.0, hip_graph: bool = False,
                 lr_schedule: str = "constant", lr_warmup_steps: int = 0, eval_hip_graph="auto"):
        self.model = model
        self.store = store
        self.optimizer = optimizer
        self.bucketer = bucketer
        self.device = torch.device(device) if device is not None else store.device
        self.grad_accum = max(1, int(grad_accum))
        self.check_sync = int(check_sync)
        self.log_every = int(log_every)
        self.step_watchdog = float(step_watchdog)
        self._watchdog = None
        self._phase = "idle"
        self.global_step = 0
        self.world = backend.size()
        self.rank = backend.rank()
        self._graphs = {}
        self.eval_hip_graph = eval_hip_graph
        self._eval_graphs = {}
        self.eval_graph_active = False  # whether the last evaluate() replayed a captured forward
        self._seed = None
        self._graph_replay = True  # tests: False = graph-mode seeding with eager kernels
        self._opt_overlap = None  # LocalOverlap (one process) | "engine" (DP ranks) | None
        self._grads_clear = False  # the last eager step's optimizer left the gradient buffer zeroed
        # learning-rate schedule: the reference's Keras Adam uses a constant rate (scripts/train.py:113); linear =
        # warmup to the base rate, then linear decay to 0 over the steps fit() is asked to run
        if lr_schedule not in ("constant", "linear"):
            raise ValueError(f"lr_schedule {lr_schedule!r}")
        self.lr_schedule = lr_schedule
        self.lr_warmup_steps = max(0, int(lr_warmup_steps))
        self.base_lr = float(getattr(optimizer, "lr", 0.0))
        self.total_steps: Optional[int] = None
        self._full_graph = False
        self._setup_opt_overlap()
        if hip_graph:
            self.enable_hip_graph()

    def _setup_opt_overlap(self) -> None:
        """Optimizer slices stepped under backward (optim/adam.py). Off: HSD_OPT_OVERLAP=0, CPU, HIP-graph mode,
        DP worlds without the native engine, and optimizers without the flat-slice API."""
        if (os.environ.get("HSD_OPT_OVERLAP", "1") == "0" or self.device.type != "cuda"
                or not hasattr(self.optimizer, "enable_overlap")):
            return
        if not getattr(self.model, "opt_overlap_safe", True):
            # the model reads weights after their gradient hook (FusedAdam.enable_overlap's invariant): no overlap
            logger.info("optimizer overlap off: %s sets opt_overlap_safe = False", type(self.model).__name__)
            return
        if self.bucketer is None and self.world == 1:
            from ..optim.adam import LocalOverlap

            self._opt_overlap = LocalOverlap(self.optimizer)
        elif self.bucketer is not None and self.bucketer.attach_optimizer(self.optimizer):
            self._opt_overlap = "engine"

    def _drop_opt_overlap(self) -> None:
        if self._opt_overlap is None:
            return
        if self._opt_overlap != "engine":
            self.store.ready_callback = None
        elif self.bucketer is not None:
            self.bucketer._on_reduced = None
        self.optimizer._ranges = []
        self._opt_overlap = None

    def enable_hip_graph(self) -> bool:
        """Replay forward + backward from captured HIP graphs (train/graph.py). Single-process GPU runs of
        models without data-dependent shapes; otherwise stays eager (returns False)."""
        if self.device.type != "cuda":
            logger.warning("--hip_graph: needs a GPU")
            return False
        if self.bucketer is not None or self.world > 1:
            # data parallel: only the whole-step graph over the native RCCL engine captures the collectives. It is
            # OPT-IN (HSD_GRAPH_DP=1): captured all-reduces + engine-stream Adam slices have been checked against
            # eager with a world-of-one communicator only (tests/test_gpu_graph.py), not on a multi-GPU node
            if not (self.bucketer is not None and self.bucketer.engine is not None and self.bucketer.overlap
                    and os.environ.get("HSD_GRAPH_FULL", "1") == "1"
                    and os.environ.get("HSD_GRAPH_DP", "0") == "1"):
                logger.warning("--hip_graph: data-parallel whole-step capture is opt-in (HSD_GRAPH_DP=1, native RCCL "
                               "engine with overlap); staying eager")
                return False
            if self.grad_accum > 1:
                logger.warning("--hip_graph: data-parallel capture covers one-micro-step optimizer steps only "
                               "(--gradient_accumulation_steps %d); staying eager", self.grad_accum)
                return False
        if not getattr(self.model, "graph_safe", True):
            logger.warning("--hip_graph: %s has data-dependent shapes; staying eager", type(self.model).__name__)
            return False
        from .graph import DeviceStepSeed

        # whole-step capture (HSD_GRAPH_FULL=1, default) for one-micro-step optimizer steps: forward, backward, the
        # overlapped optimizer slices and the weight-copy refresh in one graph; accumulation steps replay a
        # forward + backward graph per micro-step and step the optimizer eagerly
        self._full_graph = os.environ.get("HSD_GRAPH_FULL", "1") == "1" and hasattr(self.optimizer, "use_device_coef")
        self._seed = DeviceStepSeed(self.device, self.model.rng.base_seed, self.rank)
        return True

    def _full_graph_for(self, mb):
        key = ("full",) + tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(mb.items()))
        g = self._graphs.get(key)
        if g is None:
            from .graph import CapturedTrainStep

            g = self._graphs[key] = CapturedTrainStep(self, mb)
        return g

    def _graph_for(self, mb):
        key = tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(mb.items()))
        g = self._graphs.get(key)
        if g is None:
            from .graph import CapturedStep

            g = self._graphs[key] = CapturedStep(self, mb)
        return g

    # -------------------------------------------------------------------------- step
    def lr_at(self, step: int) -> float:
        """Learning rate of optimizer step ``step`` (0-based)."""
        f = 1.0
        w = self.lr_warmup_steps
        if w and step < w:
            f = (step + 1) / w
        elif self.lr_schedule == "linear" and self.total_steps:
            f = max(0.0, (self.total_steps - step) / max(1, self.total_steps - w))
        return self.base_lr * f

    def _forward_loss(self, batch):
        loss, logits = self.model(batch["input_ids"], attention_mask=batch["attention_mask"],
                                  labels=batch["labels"])
        return loss, logits

    def train_step(self, micro_batches: List[Dict[str, torch.Tensor]], meter: Optional[_Meter] = None) -> torch.Tensor:
        """One optimizer step over ``len(micro_batches)`` accumulation micro-steps."""
        self.model.train()
        if self._seed is not None and self._graph_replay and self._full_graph and len(micro_batches) == 1:
            return self._graph_step(micro_batches[0], meter)
        if self._seed is not None and self._graph_replay and self.bucketer is not None:
            raise RuntimeError("--hip_graph with data parallelism captures whole one-micro-step optimizer steps only "
                               "(gradient accumulation: run eagerly)")
        if self._seed is not None:
            # graph mode: per-site seeds fixed (step 0), the device step seed carries the step
            self._seed.set_step(self.global_step)
            self.model.rng.new_step(0)
        else:
            self.model.rng.new_step(self.global_step)
        if self._grads_clear:
            self._grads_clear = False  # the previous step's Adam cleared every gradient it read (stream-ordered)
        else:
            self.store.zero_grad()
        k = len(micro_batches)
        if self.bucketer is not None:
            self.bucketer.begin(micro_steps=k)
        if self.lr_schedule != "constant" or self.lr_warmup_steps:
            self.optimizer.lr = self.lr_at(self.global_step)
        ov = self._opt_overlap
        # the optimizer clears the gradients it consumes (no memset pass at the next step's start): eager steps with
        # the fused GPU Adam only (captured steps keep their own memset node)
        zg = self.zero_grad_in_optimizer and self.device.type == "cuda" and isinstance(self.optimizer, FusedAdam)
        if ov is not None:
            self.optimizer.begin_step(grad_scale=1.0 / (self.world * k), zero_grad=zg)
            if ov != "engine":
                ov.begin()
        loss = None
        try:
            loss = self._micro_steps(micro_batches, meter, ov, k)
        except BaseException:
            if ov is not None:
                self.optimizer.abort_step()  # the step count must not advance for a step that never happened
            self._phase = "idle"
            raise
        self._phase = "allreduce-wait"
        with prange("allreduce-wait"):
            if self.device.type == "cuda":
                ops.join_side_streams()
            if self.bucketer is not None:
                self.bucketer.finish()
            if ov is not None and ov != "engine":
                ov.join()
        self._phase = "optimizer"
        with prange("optimizer"):
            if zg:
                self.optimizer.step(grad_scale=1.0 / (self.world * k), zero_grad=True)
            else:
                self.optimizer.step(grad_scale=1.0 / (self.world * k))
        self._phase = "idle"
        self._grads_clear = zg
        self.global_step += 1
        if self.check_sync and self.global_step % self.check_sync == 0:
            if not params_in_sync(self.store):
                raise RuntimeError(f"ranks diverged at step {self.global_step} (--check_sync)")
        return loss

    def _graph_step(self, mb, meter):
        """One optimizer step as one replay of the captured whole-step graph (train/graph.py CapturedTrainStep)."""
        self._seed.set_step(self.global_step)
        self.model.rng.new_step(0)
        if self.lr_schedule != "constant" or self.lr_warmup_steps:
            self.optimizer.lr = self.lr_at(self.global_step)
        self._grads_clear = False  # the captured step keeps its own memset node and leaves gradients in place
        self._phase = "graph-step"
        with prange("graph-step"):
            loss, logits = self._full_graph_for(mb).run(mb)
        if meter is not None:
            meter.update(loss, logits, mb["labels"], static=True)
        self._phase = "idle"
        self.global_step += 1
        if self.check_sync and self.global_step % self.check_sync == 0:
            if not params_in_sync(self.store):
                raise RuntimeError(f"ranks diverged at step {self.global_step} (--check_sync)")
        return loss

    def _micro_steps(self, micro_batches, meter, ov, k):
        """Forward + backward of every accumulation micro-step (the bucket all-reduces and, with the optimizer
        overlap, the Adam slices start under the last backward)."""
        loss = None
        for i, mb in enumerate(micro_batches):
            last = i == k - 1
            if self._seed is not None and i > 0:
                # graph-mode seeding: every micro-step draws its own dropout masks (replayed graphs included)
                self._seed.set_step(self.global_step, i)
                self.model.rng.new_step(0)
            if ov is not None and ov != "engine":
                ov.sync = last  # accumulation micro-steps: gradients not final
            if self._seed is not None and self._graph_replay:
                with prange("graph-replay"):
                    loss, logits = self._graph_for(mb).run(mb)
                if meter is not None:
                    meter.update(loss, logits, mb["labels"], static=True)
                continue
            ctx = self.bucketer.no_sync() if (self.bucketer is not None and not last) else contextlib.nullcontext()
            with ctx:
                self._phase = "forward"
                with prange("forward"):
                    loss, logits = self._forward_loss(mb)
                self._phase = "backward+allreduce"
                with prange("backward+allreduce"):
                    loss.backward()
            if meter is not None:
                meter.update(loss, logits, mb["labels"])
        return loss

    # -------------------------------------------------------------------------- stall watchdog
    def _watchdog_context(self) -> str:
        last = None
        if self.bucketer is not None:
            last = getattr(self.bucketer, "last_launched", None)
        return (f"phase {self._phase}; last launched gradient bucket {last if last is not None else '-'}"
                + (f" of {len(self.bucketer.buckets)}" if self.bucketer is not None else ""))

    def start_watchdog(self) -> None:
        """--step_watchdog S: a monitor thread ends the process if no step completes (on the device) for S
        seconds (train/watchdog.py); the launcher then tears the group down."""
        if self.step_watchdog > 0 and self._watchdog is None:
            from .watchdog import StepWatchdog

            self._watchdog = StepWatchdog(self.step_watchdog, rank=self.rank, describe=self._watchdog_context).start()

    def stop_watchdog(self) -> None:
        if self._watchdog is not None:
            self._watchdog.stop()
            self._watchdog = None

    # -------------------------------------------------------------------------- fit
    def fit(self, loader, epochs: int, callbacks: Iterable = (), verbose: bool = True,
            max_steps: Optional[int] = None, initial_epoch: int = 0) -> History:
        """Keras ``fit(epochs=..., initial_epoch=...)``: runs epochs ``initial_epoch .. epochs-1`` (a resumed
        run continues the epoch count of its checkpoint instead of training ``epochs`` more)."""
        hist = History()
        callbacks = list(callbacks)
        per_epoch = len(loader) // self.grad_accum
        if max_steps:
            per_epoch = min(per_epoch, max_steps)
        self.total_steps = self.global_step + per_epoch * max(0, epochs - int(initial_epoch))
        for cb in callbacks:
            cb.on_train_begin(self)
        self.start_watchdog()
        try:
            self._fit_epochs(loader, epochs, callbacks, verbose, max_steps, initial_epoch, hist)
        finally:
            self.stop_watchdog()
        for cb in callbacks:
            cb.on_train_end(self)
        return hist

    def _fit_epochs(self, loader, epochs, callbacks, verbose, max_steps, initial_epoch, hist) -> None:
        wd = self._watchdog
        for epoch in range(int(initial_epoch), epochs):
            if hasattr(loader, "sampler"):
                loader.sampler.set_epoch(epoch)
            meter = _Meter(self.device)
            nsteps = len(loader) // self.grad_accum
            if max_steps:
                nsteps = min(nsteps, max_steps)
            t0 = time.time()
            it = iter(loader)
            for step in range(nsteps):
                mbs = [next(it) for _ in range(self.grad_accum)]
                if wd is not None:
                    wd.step_begin(self.global_step)
                self.train_step(mbs, meter)
                if wd is not None:
                    wd.step_end(self.global_step - 1, self.device)
                if verbose and self.rank == 0 and self.log_every and (step + 1) % self.log_every == 0:
                    r = meter.result(global_=False)
                    logger.info("epoch %d step %d/%d - loss: %.4f - sparse_categorical_accuracy: %.4f - %.1f ms/step",
                                epoch + 1, step + 1, nsteps, r["loss"], r["sparse_categorical_accuracy"],
                                (time.time() - t0) * 1e3 / (step + 1))
                for cb in callbacks:
                    cb.on_batch_end(self, step)
            for _ in it:  # drain the prefetch thread
                pass
            logs = meter.result(global_=True)
            hist.append(epoch, logs)
            if verbose and self.rank == 0:
                logger.info("Epoch %d/%d - %.1fs - loss: %.4f - sparse_categorical_accuracy: %.4f", epoch + 1, epochs,
                            time.time() - t0, logs["loss"], logs["sparse_categorical_accuracy"])
            for cb in callbacks:
                cb.on_epoch_end(self, epoch, logs)

    # -------------------------------------------------------------------------- evaluate
    def _eval_graph_wanted(self, tokens: int) -> bool:
        """``eval_hip_graph``: True / False as given; ``auto`` = replay captured eval forwards for batches of at most
        HSD_EVAL_GRAPH_MAX_TOKENS (16,384) tokens on the GPU, where one forward is a few hundred short launches."""
        flag = self.eval_hip_graph
        if self.device.type != "cuda" or not getattr(self.model, "graph_safe", True) or not ops.hip_active(self.device):
            return False
        if flag != "auto":
            return bool(flag)
        return tokens <= int(os.environ.get("HSD_EVAL_GRAPH_MAX_TOKENS", "16384"))

    def _eval_forward(self, b):
        """(loss, logits, static): a captured replay when the eval graph is on for this shape, else eager."""
        ids = b["input_ids"]
        if self._eval_graph_wanted(ids.numel()):
            key = tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(b.items()) if torch.is_tensor(v))
            g = self._eval_graphs.get(key)
            if g is None and key not in self._eval_graphs:
                from .graph import CapturedEval

                try:
                    g = CapturedEval(self, b)
                except Exception as e:  # an op that cannot be captured: this shape stays eager (loudly)
                    logger.warning("eval graph capture failed for shape %s (%s): eager forward", tuple(ids.shape), e)
                    g = None
                self._eval_graphs[key] = g
            if g is not None:
                self.eval_graph_active = True
                loss, logits = g.run(b)
                return loss, logits, True
        loss, logits = self._forward_loss(b)
        return loss, logits, False

    @torch.no_grad()
    def evaluate(self, loader, max_steps: Optional[int] = None) -> Dict[str, float]:
        self.model.eval()
        self.eval_graph_active = False
        meter = _Meter(self.device)
        for i, b in enumerate(loader):
            if max_steps and i >= max_steps:
                continue  # drain
            if b.get("num_valid", 1) == 0:
                continue  # a shard's tail made only of padding rows
            loss, logits, static = self._eval_forward(b)
            meter.update(loss, logits, b["labels"], static=static)
            if self.rank == 0 and self.log_every and (i + 1) % (self.log_every * 20) == 0:
                # progress only (Keras' evaluate progress bar): host-side count, no device sync
                logger.info("evaluate: %d/%d batches issued", i + 1, len(loader))
        return meter.result(global_=True)
