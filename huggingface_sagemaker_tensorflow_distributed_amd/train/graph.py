"""HIP-graph capture of the training step's forward + backward (SURVEY.md §2.4 'XLA / graph compilation
-> HIP graphs for the step', §7.4 hard part 4 'host launch overhead').

A BERT step is ~25 kernels per layer (several hundred launches per step); at small per-GPU batches the
host cannot issue them as fast as the GPU retires them. :class:`CapturedStep` records forward + loss +
backward ONCE into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) over static input buffers and then
replays it: one launch per micro-step. The optimizer (one fused Adam + one batched Wᵀ refresh) stays
eager — it is two launches and its step-dependent scalars live on the host.

What makes a replay a *fresh* step:

* inputs are copied into the static buffers (``copy_`` on the stream, no host sync);
* dropout: every kernel's per-call-site seed is baked into the graph, and each step XORs a device-side
  step seed into it (``_C.set_dropout_device_seed``; common.h ``DropoutParams::dev_seed``), so the masks
  change every step without re-capture. Eager steps of a graph-enabled trainer use the same device
  seed, so eager and replayed steps draw identical masks for the same step index;
* gradients: the flat ``main_grad`` buffer is zeroed before the replay (kernels accumulate into it).

Limits: fixed batch shape per captured graph (a new shape captures a new graph), models without data-dependent
shapes (the MLM head's masked-token gather syncs the host: eager only). Data-parallel steps are captured whole only
on request (HSD_GRAPH_DP=1, :class:`CapturedTrainStep` with the native RCCL engine's bucket all-reduces inside the
graph); by default they keep the eager path.
"""
from __future__ import annotations

import gc
import logging
from typing import Dict

import torch

from ..ops.rng import mix32_int

logger = logging.getLogger(__name__)


class _NoGC:
    """Python's cyclic collector stays off while a graph is captured: a collection frees whatever cycles are due, and
    a finaliser that synchronises a stream or frees device memory (an RCCL communicator's teardown) is an unsafe call
    inside a capture (it invalidates it; the replay of such a graph faulted on the host). torch.cuda.graph collects
    right before the capture begins."""

    def __enter__(self):
        self.was = gc.isenabled()
        gc.disable()
        return self

    def __exit__(self, *exc):
        if self.was:
            gc.enable()
        return False


def step_seed(base_seed: int, rank: int, step: int, micro: int = 0):
    """Two 32-bit words of the device step seed for accumulation micro-step ``micro`` of optimizer step ``step``."""
    a = mix32_int((base_seed ^ 0x2545F491) & 0xFFFFFFFF)
    b = mix32_int(a ^ ((step * 0x9E3779B9 + rank * 0x7F4A7C15 + micro * 0x85EBCA6B) & 0xFFFFFFFF))
    c = mix32_int(b ^ 0x68E31DA4)
    return b, c


class DeviceStepSeed:
    """The process-wide device step seed (int32 [2]) read by every dropout kernel."""

    def __init__(self, device, base_seed: int, rank: int):
        from ..ops import hip

        self.t = torch.zeros(2, dtype=torch.int32, device=device)
        self.base_seed, self.rank = int(base_seed), int(rank)
        hip._C.set_dropout_device_seed(self.t)

    def set_step(self, step: int, micro: int = 0) -> None:
        lo, hi = step_seed(self.base_seed, self.rank, step, micro)
        # stream-ordered fills (the value travels as a kernel argument: no host buffer the GPU could
        # read after the host moved on to the next step); int32 view of the uint32 words
        self.t[0].fill_(lo - (1 << 32) if lo >= 1 << 31 else lo)
        self.t[1].fill_(hi - (1 << 32) if hi >= 1 << 31 else hi)

    def close(self) -> None:
        from ..ops import hip

        hip._C.set_dropout_device_seed(None)


class CapturedStep:
    """forward + loss + backward of ``trainer`` for batches shaped like ``example``, as one graph."""

    def __init__(self, trainer, example: Dict[str, torch.Tensor], warmup: int = 2):
        self.trainer = trainer
        self.static = {k: v.clone() for k, v in example.items()}
        model, store = trainer.model, trainer.store
        model.train()
        # warm up on a side stream (kernel/workspace first-use allocations, lazy caches) — not captured; no
        # readiness callbacks (an optimizer step may already have begun: its slices must not see warm-up gradients)
        saved = store.grad.clone()  # earlier micro-steps of this optimizer step (gradient accumulation)
        s = torch.cuda.Stream(device=trainer.device)
        s.wait_stream(torch.cuda.current_stream(trainer.device))
        cb, store.ready_callback = store.ready_callback, None
        try:
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    model.rng.new_step(0)
                    store.zero_grad()
                    loss, _ = trainer._forward_loss(self.static)
                    loss.backward()
        finally:
            store.ready_callback = cb
        torch.cuda.current_stream(trainer.device).wait_stream(s)
        torch.cuda.synchronize(trainer.device)
        store.grad.copy_(saved)  # the warm-up overwrote main_grad
        del saved
        self.graph = torch.cuda.CUDAGraph()
        cb, store.ready_callback = store.ready_callback, None  # no optimizer slices inside a fwd+bwd-only graph
        from ..ops import hip

        try:
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"), _NoGC():
                hip.begin_capture(torch.cuda.current_stream(trainer.device))
                model.rng.new_step(0)  # per-site seeds fixed; the device step seed varies per replay
                self.loss, self.logits = trainer._forward_loss(self.static)
                self.loss.backward()
                hip.join_side_streams()
        finally:
            hip.end_capture()
            store.ready_callback = cb
        torch.cuda.synchronize(trainer.device)
        logger.info("captured training step graph for batch shape %s", tuple(example["input_ids"].shape))

    def run(self, batch: Dict[str, torch.Tensor]):
        """Copy ``batch`` into the static inputs and replay (gradients ACCUMULATE into main_grad)."""
        for k, v in batch.items():
            self.static[k].copy_(v, non_blocking=True)
        self.graph.replay()
        return self.loss, self.logits


class CapturedEval:
    """The eval-mode forward + loss + fused metric counts of ``trainer`` for batches shaped like ``example``, as one
    graph: the reference's ``model.evaluate`` at ``eval_batch_size`` 2 (``launch.py:16``, ``scripts/train.py:170``) is
    12,500 forwards of 2 sequences, each a few hundred short kernels -- launch-bound when issued one by one. No dropout
    (eval mode: no seeds), no autograd (``no_grad``): nothing but the static inputs changes between replays."""

    def __init__(self, trainer, example: Dict[str, torch.Tensor], warmup: int = 1):
        self.trainer = trainer
        self.static = {k: v.clone() for k, v in example.items() if torch.is_tensor(v)}
        model = trainer.model
        model.eval()
        dev = trainer.device
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(s):
            for _ in range(warmup):  # first-use workspaces / lazy caches, outside the capture
                trainer._forward_loss(self.static)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph, capture_error_mode="thread_local"), _NoGC():
            self.loss, self.logits = trainer._forward_loss(self.static)
        torch.cuda.synchronize(dev)
        logger.info("captured eval forward graph for batch shape %s", tuple(example["input_ids"].shape))

    def run(self, batch: Dict[str, torch.Tensor]):
        for k, v in self.static.items():
            v.copy_(batch[k], non_blocking=True)
        self.graph.replay()
        return self.loss, self.logits


class CapturedTrainStep:
    """The WHOLE training step as one graph: gradient zeroing, forward, loss, backward, the optimizer slices stepped
    under backward (one process: optim/adam.py LocalOverlap, a side-stream branch of the graph per slice, forked when
    the slice's last gradient is queued; data parallel: the native RCCL engine's bucket all-reduces, each followed by
    its Adam slice on the engine stream), the remaining slices and the Wᵀ / fp8 weight-copy refresh.

    Adam's per-step scalars (bias-corrected step, ε, grad scale, lr·wd) are read from a device tensor
    (``FusedAdam.use_device_coef``) that :meth:`run` refreshes before each replay, as the dropout step seed is; the
    Python-side optimizer bookkeeping that ran once during capture is replayed by hand (step count). Capturing
    runs no kernel, so it changes no weight; the forward + backward warm-up before it (lazy workspaces, first-use
    allocations) leaves the gradients zeroed."""

    def __init__(self, trainer, example: Dict[str, torch.Tensor], warmup: int = 2):
        self.trainer = trainer
        self.static = {k: v.clone() for k, v in example.items()}
        model, store, opt = trainer.model, trainer.store, trainer.optimizer
        model.train()
        s = torch.cuda.Stream(device=trainer.device)
        s.wait_stream(torch.cuda.current_stream(trainer.device))
        cb, store.ready_callback = store.ready_callback, None
        try:
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    model.rng.new_step(0)
                    store.zero_grad()
                    loss, _ = trainer._forward_loss(self.static)
                    loss.backward()
        finally:
            store.ready_callback = cb
        torch.cuda.current_stream(trainer.device).wait_stream(s)
        torch.cuda.synchronize(trainer.device)
        store.zero_grad()
        opt.use_device_coef()
        ov = trainer._opt_overlap
        buck = trainer.bucketer
        eng = buck.engine if buck is not None else None
        gscale = 1.0 / trainer.world
        from ..ops import hip

        self.graph = torch.cuda.CUDAGraph()
        step0 = opt.step_count
        try:
            with opt.capturing(), torch.cuda.graph(self.graph, capture_error_mode="thread_local"), _NoGC():
                cap = torch.cuda.current_stream(trainer.device)  # the capture stream
                # the weight-gradient side stream runs as a branch of the graph (ops/hip.py begin_capture), as in
                # eager steps: captured sequentially it made the replay slower than eager (round 3)
                hip.begin_capture(cap)
                store.zero_grad()
                model.rng.new_step(0)
                if eng is not None:
                    # data parallel: the bucket all-reduces (and, with the engine overlap, each bucket's Adam slice
                    # on the engine stream) are captured too -- the engine forks its stream from the capture stream
                    eng.set_caller_stream(cap.cuda_stream)
                    buck.begin(micro_steps=1)
                if ov is not None:
                    if ov != "engine":
                        ov.parent = cap
                    opt.begin_step(grad_scale=gscale)
                    if ov != "engine":
                        ov.begin()
                self.loss, self.logits = trainer._forward_loss(self.static)
                self.loss.backward()
                hip.join_side_streams()
                if buck is not None:
                    buck.finish()
                if ov is not None and ov != "engine":
                    ov.join()
                opt.step(grad_scale=gscale)
        finally:
            hip.end_capture()
            if ov is not None and ov != "engine":
                ov.parent = None
            if eng is not None:
                eng.set_caller_stream(0)
        opt.step_count = step0  # begin_step / step advanced it once during capture; each replay advances it
        torch.cuda.synchronize(trainer.device)
        self.gscale = gscale
        logger.info("captured whole training step graph (optimizer %s) for batch shape %s",
                    "overlapped" if ov is not None else "after backward", tuple(example["input_ids"].shape))

    def run(self, batch: Dict[str, torch.Tensor]):
        """Copy ``batch`` in, set this step's optimizer scalars, replay: one complete optimizer step."""
        for k, v in batch.items():
            self.static[k].copy_(v, non_blocking=True)
        self.trainer.optimizer.prepare_device_step(self.gscale)
        self.graph.replay()
        return self.loss, self.logits
