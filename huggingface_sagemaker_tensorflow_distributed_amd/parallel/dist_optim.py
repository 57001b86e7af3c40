"""``hvd.DistributedOptimizer``: an optimizer object whose ``step()`` applies the rank-averaged gradient.

Reference: ``optimizer = hvd.DistributedOptimizer(optimizer)`` (``scripts/train.py:114``) wraps the Keras Adam so
that every ``apply_gradients`` uses the all-reduced gradient; Horovod's ``backward_passes_per_step=k`` accumulates k
local backward passes per parameter before it all-reduces, and ``compression=hvd.Compression.fp16`` sets the wire
dtype.

Here the wrapped object is a :class:`optim.FusedAdam` over a :class:`FlatParamStore`; the collective work is a
:class:`GradBucketer` (RCCL engine buckets fired from the store's post-accumulate hooks, i.e. overlapped with
backward). The plain PyTorch loop works unchanged::

    opt = hvd.DistributedOptimizer(FusedAdam(store, lr=5e-5), compression=hvd.Compression.fp16)
    for batch in loader:
        opt.zero_grad()
        loss.backward()          # buckets all-reduce as their gradients complete
        opt.step()               # waits for the buckets, Adam with grad_scale = 1 / (world x k)

The Trainer (``train/trainer.py``) drives the same bucketer directly and adds the optimizer-under-backward overlap;
this wrapper is the API-compatible path for user code written against Horovod.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

from . import backend
from .ddp import GradBucketer


class DistributedOptimizer:
    def __init__(self, optimizer, store=None, bucket_mb: Optional[float] = None, compression: str = "none",
                 backward_passes_per_step: int = 1, group=None):
        if backward_passes_per_step < 1:
            raise ValueError("backward_passes_per_step must be >= 1")
        self.optimizer = optimizer
        self.store = store if store is not None else optimizer.store
        self.world = backend.size()
        self.backward_passes_per_step = int(backward_passes_per_step)
        self.bucketer = (GradBucketer(self.store, bucket_mb=bucket_mb, compression=compression, group=group)
                         if self.world > 1 else None)
        self._passes: List[int] = [0] * len(self.store.segments)
        self._begun = False
        # per-parameter backward-pass counter in front of the bucketer (Horovod's backward_passes_per_step): a
        # parameter's k-th gradient is the one that marks it ready for its bucket
        self.store.ready_callback = self._on_ready

    # ------------------------------------------------------------------ hooks
    def _begin(self) -> None:
        if self.bucketer is not None:
            self.bucketer.begin(micro_steps=self.backward_passes_per_step)
        self._passes = [0] * len(self._passes)
        self._begun = True

    def _on_ready(self, i: int) -> None:
        if not self._begun:
            self._begin()
        self._passes[i] += 1
        if self._passes[i] > self.backward_passes_per_step and self.bucketer is not None:
            # Horovod raises here too: the bucket holding this gradient was already reduced, so the extra pass would
            # be applied on this rank only and the replicas would diverge. A world of one has no bucket (Horovod
            # registers no hooks at size() == 1): extra local passes just accumulate
            raise RuntimeError(
                f"parameter {i} received {self._passes[i]} gradients before step(), more than "
                f"backward_passes_per_step={self.backward_passes_per_step}")
        if self._passes[i] == self.backward_passes_per_step and self.bucketer is not None:
            self.bucketer.mark_ready(i)

    # ------------------------------------------------------------------ optimizer API
    def zero_grad(self, set_to_none: bool = False) -> None:  # noqa: ARG002 - flat buffer: always zeroed in place
        self.store.zero_grad()
        self._begin()

    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if not self._begun:
            self._begin()
        if self.store.device.type == "cuda":
            from ..ops import hip

            hip.join_side_streams()
        if self.bucketer is not None:
            self.bucketer.finish()  # launches buckets no gradient reached, waits for all
        self.optimizer.step(grad_scale=1.0 / (self.world * self.backward_passes_per_step))
        self._begun = False
        return loss

    def synchronize(self) -> None:
        """Horovod's ``optimizer.synchronize()``: finish the outstanding all-reduces without stepping."""
        if self.bucketer is not None:
            self.bucketer.finish()

    @contextlib.contextmanager
    def skip_synchronize(self):
        yield

    def state_dict(self) -> dict:
        return self.optimizer.state_dict()

    def load_state_dict(self, sd: dict) -> None:
        self.optimizer.load_state_dict(sd)

    def __getattr__(self, name):  # lr, step_count, exp_avg, ... of the wrapped optimizer
        if name == "optimizer":
            raise AttributeError(name)
        return getattr(self.optimizer, name)

    def __setattr__(self, name, value):
        if name == "lr" and "optimizer" in self.__dict__:
            self.optimizer.lr = value
        else:
            object.__setattr__(self, name, value)
