"""Fused Adam / AdamW over the flat parameter store — one kernel launch per step.

Reference optimizer: ``tf.keras.optimizers.Adam(learning_rate)`` (``scripts/train.py:113``,
``scripts/singe_node_train.py:78``) — TF 2.4 Keras defaults β1=0.9, β2=0.999, ε=1e-7, no weight decay,
and the ε-hat update::

    lr_t = lr·√(1-β2ᵗ)/(1-β1ᵗ);  m = β1 m + (1-β1) g;  v = β2 v + (1-β2) g²;  θ -= lr_t·m/(√v + ε)

PyTorch's form divides √v by √(1-β2ᵗ) before adding ε; both are ``θ -= step·m/(√v + ε_eff)`` with
``ε_eff = ε`` (keras) or ``ε·√(1-β2ᵗ)`` (torch), so one kernel serves both (``eps_mode``).
The DP ``1/N`` gradient average (``hvd.DistributedOptimizer`` semantics) and the optional
gradient-accumulation ``1/k`` are folded into ``grad_scale``; with bf16 compute the kernel also
writes the bf16 weight copy the next forward reads (no separate cast pass).

Overlap with backward (:meth:`FusedAdam.enable_overlap`): the update is elementwise, so a contiguous slice of the
flat buffers can be stepped as soon as its gradients are final. The store is laid out in backward order, so
the slices complete front-to-back while the rest of backward still runs: one process runs each slice's Adam on
a side stream the moment its last gradient is queued; data-parallel ranks run it on the RCCL engine's stream
right after the slice's bucket all-reduce. The memory-bound update then shares the GPU with the compute-bound
backward GEMMs instead of following them (the bert-large optimizer pass moves ~10 GB per step). What is left
at ``step()`` is the join, the slices no gradient reached, and the batched Wᵀ refresh.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Callable, Iterable, List, Optional, Tuple

import torch

from ..parallel.flat_params import ALIGN, FlatParamStore


class FusedAdam:
    # overlapped steps re-quantise each slice's fp8 weights right after its update (False: one pass at the end; A/B)
    per_slice_fp8 = True

    def __init__(self, store: FlatParamStore, lr: float = 1e-3, betas=(0.9, 0.999), eps: Optional[float] = None,
                 weight_decay: float = 0.0, eps_mode: str = "keras", decoupled: bool = True):
        if eps_mode not in ("keras", "torch"):
            raise ValueError(eps_mode)
        self.store = store
        self.lr = float(lr)
        self.beta1, self.beta2 = map(float, betas)
        self.eps = float(eps if eps is not None else (1e-7 if eps_mode == "keras" else 1e-8))
        self.eps_mode = eps_mode
        self.weight_decay = float(weight_decay)
        self.decoupled = decoupled
        self.step_count = 0
        self.exp_avg = torch.zeros_like(store.master)
        self.exp_avg_sq = torch.zeros_like(store.master)
        self._decay_mask = store.decay_block_mask(ALIGN) if weight_decay else None
        self.dcoef: Optional[torch.Tensor] = None  # device-side step scalars (HIP-graph replays), see use_device_coef
        self._capturing = False  # dcoef is handed to the kernel only while a whole-step graph is being captured

    # --------------------------------------------------------------------------
    def state_tensors(self) -> List[torch.Tensor]:
        return [self.exp_avg, self.exp_avg_sq]

    def state_dict(self) -> dict:
        return {"step": self.step_count, "exp_avg": self.exp_avg.cpu(), "exp_avg_sq": self.exp_avg_sq.cpu(),
                "lr": self.lr, "betas": (self.beta1, self.beta2), "eps": self.eps, "eps_mode": self.eps_mode,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd: dict) -> None:
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"].to(self.exp_avg.device))
        self.exp_avg_sq.copy_(sd["exp_avg_sq"].to(self.exp_avg_sq.device))

    def _coeffs(self):
        t = self.step_count
        bc1 = 1.0 - self.beta1 ** t
        bc2 = 1.0 - self.beta2 ** t
        step = self.lr * math.sqrt(bc2) / bc1
        eps_eff = self.eps if self.eps_mode == "keras" else self.eps * math.sqrt(bc2)
        return step, eps_eff

    # -------------------------------------------------------------------------- device-side coefficients
    def use_device_coef(self) -> torch.Tensor:
        """The fp32 [4] device tensor (step, eps, grad_scale, lr*wd) that Adam launches CAPTURED into a HIP graph of
        the whole training step read instead of kernel arguments, so replays run with each step's bias correction
        and learning rate (train/graph.py). :meth:`prepare_device_step` fills it before a replay. Only launches
        issued inside :meth:`capturing` read it; eager steps always pass their own scalars."""
        if self.dcoef is None:
            self.dcoef = torch.zeros(4, dtype=torch.float32, device=self.store.master.device)
        return self.dcoef

    @contextlib.contextmanager
    def capturing(self):
        """Scope of a whole-step graph capture: Adam launches inside it take their scalars from :attr:`dcoef`."""
        self.use_device_coef()
        self._capturing = True
        try:
            yield
        finally:
            self._capturing = False

    def _kernel_coef(self) -> Optional[torch.Tensor]:
        return self.dcoef if self._capturing else None

    def prepare_device_step(self, grad_scale: float) -> None:
        """Advance the step count and write this step's scalars to :attr:`dcoef` (stream-ordered H2D copy of a
        fresh host tensor: the host may move on at once)."""
        self.step_count += 1
        step, eps_eff = self._coeffs()
        self.dcoef.copy_(torch.tensor([step, eps_eff, float(grad_scale), self.lr * self.weight_decay],
                                      dtype=torch.float32), non_blocking=True)

    # -------------------------------------------------------------------------- overlap with backward
    def enable_overlap(self, ranges: List[Tuple[int, int]], on_ready: Optional[Callable] = None) -> None:
        """Step the flat-buffer slices ``ranges`` (64-aligned, backward order) as their gradients complete.

        INVARIANT (the overlap is correct only under it): every kernel that READS a parameter -- its bf16 copy, its
        Wᵀ / fp8 copies -- is queued before that parameter's post-accumulate hook fires. Autograd runs the hook after
        the last node that used the parameter, and the HIP backward kernels read weights inside those nodes, so this
        holds for the model code here; it would NOT hold for activation recompute (a re-run forward reads weights
        after their hook) or a head that reads weights outside autograd after the hook. A model that breaks it sets
        ``opt_overlap_safe = False`` and the Trainer then steps the optimizer once after backward.

        ``on_ready``: the store-readiness callback to install (one process); data-parallel ranks call
        :meth:`step_range` from the bucketer instead."""
        self._ranges = list(ranges)
        self._done = [False] * len(self._ranges)
        self._began = False
        # each slice's Wᵀ copies are refreshed right after its update (fp8 weight copies, which need the whole
        # step's amax, are still re-quantised once at the end)
        self._tsub = self.store.transposed_subsets(self._ranges) if self.store.master.is_cuda else None
        # ... and each slice's fp8 weight copies right after that (fp8 runs): the per-weight amax / quantise passes
        # leave the end of the step, where they ran alone (~0.5 ms per roberta-large step)
        self._f8sub = self.store.fp8_subsets(self._ranges) if self._tsub is not None and self.per_slice_fp8 else None
        if on_ready is not None:
            self.store.ready_callback = on_ready

    @property
    def overlap_enabled(self) -> bool:
        return bool(getattr(self, "_ranges", None))

    def begin_step(self, grad_scale: float, zero_grad: bool = False) -> None:
        """Fix this step's coefficients before backward (the slices are stepped during it). ``zero_grad``: each slice's
        Adam also clears the gradients it read (:meth:`step`)."""
        self.step_count += 1
        step, eps_eff = self._coeffs()
        self._coef = (step, eps_eff, float(grad_scale))
        self._zero = bool(zero_grad) and self.store.grad.is_cuda
        self._done = [False] * len(self._ranges)
        self._began = True

    def abort_step(self) -> None:
        """Undo :meth:`begin_step` when the step fails before :meth:`step` (an exception in backward, an OOM at an
        auto-planned batch): the bias-correction step count must not drift by one per failed step. Slices already
        stepped under the failed backward cannot be undone; the caller is expected to stop or restore a checkpoint."""
        if getattr(self, "_began", False):
            self.step_count -= 1
            self._began = False

    @torch.no_grad()
    def step_range(self, b: int) -> None:
        """Adam on slice ``b`` on the CURRENT stream (the caller orders it after the slice's gradients)."""
        if not self._began or self._done[b]:
            return
        from ..ops import hip

        st, e = self._ranges[b]
        s = self.store
        step, eps_eff, gscale = self._coef
        out, out_lo = s.adam_outputs(st, e)
        dm = self._decay_mask[st // ALIGN:(e + ALIGN - 1) // ALIGN] if self._decay_mask is not None else None
        hip.adam_step(s.master[st:e], self.exp_avg[st:e], self.exp_avg_sq[st:e], s.grad[st:e], out, dm, step,
                      eps_eff, self.beta1, self.beta2, gscale, self.lr * self.weight_decay, self._kernel_coef(), out_lo,
                      zero_grad=getattr(self, "_zero", False))
        if self._tsub is not None:
            s.refresh_transposed_subset(self._tsub[b])
        if self._f8sub is not None:
            s.refresh_fp8_subset(self._f8sub[b])
        self._done[b] = True

    @torch.no_grad()
    def _finish_overlapped(self, grad_scale: float) -> None:
        from ..ops import hip

        if abs(grad_scale - self._coef[2]) > 1e-12 * max(1.0, abs(grad_scale)):
            raise RuntimeError("FusedAdam: grad_scale changed between begin_step and step")
        hip.join_side_streams()
        for b in range(len(self._ranges)):  # slices no gradient reached (unused parameters)
            self.step_range(b)
        self._began = False
        self._zero = False
        if self._tsub is None:
            self.store.refresh_transposed()
        elif self._f8sub is not None:
            self.store.finish_fp8_step()
        else:
            self.store.refresh_fp8()

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, zero_grad: bool = False) -> None:
        """``zero_grad`` (GPU): the kernel clears each gradient after reading it, so the caller (the Trainer) can skip
        its next :meth:`FlatParamStore.zero_grad` -- the memset pass over the whole gradient buffer moves into the
        optimizer's own pass (which, overlapped with backward, runs under the weight-gradient GEMMs). With the overlap,
        :meth:`begin_step` decides it."""
        if getattr(self, "_began", False):
            self._finish_overlapped(grad_scale)
            return
        self.step_count += 1
        step, eps_eff = self._coeffs()
        s = self.store
        write_compute = s.compute is not s.master
        if s.master.is_cuda:
            from ..ops import hip

            hip.join_side_streams()  # weight gradients may still be in flight on the wgrad stream
            out, out_lo = s.adam_outputs(0, s.numel)
            hip.adam_step(s.master, self.exp_avg, self.exp_avg_sq, s.grad, out,
                          self._decay_mask, step, eps_eff, self.beta1, self.beta2, float(grad_scale),
                          self.lr * self.weight_decay, self._kernel_coef(), out_lo, zero_grad=zero_grad)
            s.refresh_transposed()
            return
        # reference path (CPU): identical math on flat buffers
        g = s.grad.to(torch.float32) * grad_scale
        if self.weight_decay:
            wd = self._decay_mask.repeat_interleave(ALIGN)[: s.numel].to(torch.float32)
            s.master.mul_(1.0 - self.lr * self.weight_decay * wd)
        self.exp_avg.mul_(self.beta1).add_(g, alpha=1.0 - self.beta1)
        self.exp_avg_sq.mul_(self.beta2).addcmul_(g, g, value=1.0 - self.beta2)
        s.master.addcdiv_(self.exp_avg, self.exp_avg_sq.sqrt().add_(eps_eff), value=-step)
        if write_compute:
            s.compute.copy_(s.master)


def plan_ranges(store: FlatParamStore, bucket_mb: float) -> Tuple[List[Tuple[int, int]], List[int]]:
    """Contiguous slices of ~``bucket_mb`` of gradients over whole segments, and each parameter's slice."""
    limit = int(bucket_mb * (1 << 20)) // store.grad.element_size()
    ranges, owner, start = [], [0] * len(store.segments), 0
    for i, _seg in enumerate(store.segments):
        owner[i] = len(ranges)
        end = store.segments[i + 1].offset if i + 1 < len(store.segments) else store.numel
        if end - start >= limit or i + 1 == len(store.segments):
            ranges.append((start, end))
            start = end
    return ranges, owner


class LocalOverlap:
    """One-process driver of :meth:`FusedAdam.enable_overlap`: counts each slice's ready gradients (the store's
    post-accumulate hooks) and, when the last one is queued, runs the slice's Adam on a side stream that first
    waits for everything queued so far on the compute (and wgrad) streams."""

    # False: every slice records its own event on the compute stream (the round-5 behaviour), for A/B runs
    defer_to_fork = True

    def __init__(self, opt: FusedAdam, bucket_mb: Optional[float] = None):
        store = opt.store
        # 16 MiB slices: bert-large S=512 B=8 +0.6 % over 32 (more of the optimizer under the backward), the headline
        # neutral (profiles/opt_slice_size_ab_r4.log)
        mb = bucket_mb if bucket_mb else float(os.environ.get("HSD_OPT_BUCKET_MB", "16"))
        self.ranges, self.owner = plan_ranges(store, mb)
        self.count = [0] * len(self.ranges)
        for o in self.owner:
            self.count[o] += 1
        self.pending = list(self.count)
        self.opt = opt
        self.stream = torch.cuda.Stream(device=store.device)
        self.sync = True
        # the stream the backward kernels are queued on, when it is not the hook thread's current stream: a HIP
        # graph capture (the capture stream; train/graph.py). Post-accumulate hooks of gradients the HIP backward
        # writes into main_grad itself run on autograd's thread with no producer stream (its current stream is the
        # device default), so a slice's fork must name the stream the gradients were really queued on.
        self.parent: Optional[torch.cuda.Stream] = None
        # contention emulation (tools/contention_ab.py): before each of the first HSD_HOG_POINTS slices of a step,
        # hold HSD_HOG_CUS whole CUs for HSD_HOG_US us on the slice stream -- what a data-parallel rank's RCCL
        # all-reduce kernels do beside its backward GEMMs -- so one GPU measures the persistent GEMMs under it
        self._hog = (int(os.environ.get("HSD_HOG_CUS", "0")), float(os.environ.get("HSD_HOG_US", "400")),
                     int(os.environ.get("HSD_HOG_POINTS", "7")))
        self._hogs = 0
        # slices whose gradients are final, waiting for the next weight-gradient fork (eager steps): a slice must
        # follow every compute-stream kernel that wrote its gradients or READ its weights (the block's last dgrad is
        # queued after the block's last fork), and the NEXT fork's side-stream position is after all of them. Ordering
        # the slice behind that position (an event recorded on the side stream) instead of recording an event on the
        # compute stream per slice takes ~3 us per slice off the compute stream's critical path (tools/fork_cost.py).
        self._deferred: List[int] = []
        self._forked = False  # a weight-gradient fork happened in this backward
        from ..ops import hip

        if self._on_fork not in hip._FORK_LISTENERS:
            hip._FORK_LISTENERS.append(self._on_fork)
        opt.enable_overlap(self.ranges, on_ready=self.mark_ready)

    def begin(self) -> None:
        self.pending = list(self.count)
        self.sync = True
        self._hogs = 0
        self._deferred = []
        self._forked = False

    def _launch(self, blocks: List[int]) -> None:
        with torch.cuda.stream(self.stream):
            for b in blocks:
                if self._hog[0] > 0 and self._hogs < self._hog[2]:
                    from ..ops import hip

                    self._hogs += 1
                    hip._C.cu_hog(self._hog[0], self._hog[1])
                self.opt.step_range(b)

    def _on_fork(self, side) -> None:
        """A weight-gradient fork just made ``side`` wait for the compute stream: the deferred slices follow it."""
        if side.device != self.stream.device:
            return
        self._forked = True
        if self._deferred:
            from ..ops import hip

            hip.stream_wait(self.stream, side)
            blocks, self._deferred = self._deferred, []
            self._launch(blocks)

    def mark_ready(self, i: int) -> None:
        if not self.sync:  # accumulation micro-step: gradients are not final yet
            return
        b = self.owner[i]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            if self.parent is None and self._forked and self.defer_to_fork:
                self._deferred.append(b)  # launched behind the next weight-gradient fork (or at join)
                return
            from ..ops import hip

            cur = self.parent if self.parent is not None else torch.cuda.current_stream(self.stream.device)
            hip.stream_wait(self.stream, cur)
            side = hip.side_stream(self.stream.device)
            if side is not None and hip.side_stream_waitable():
                hip.stream_wait(self.stream, side)
            self._launch([b])

    def join(self) -> None:
        from ..ops import hip

        cur = torch.cuda.current_stream(self.stream.device)
        if self._deferred:
            # slices ready after the backward's last fork: behind the compute stream, which has joined the side
            # stream by now (Trainer.train_step joins the side streams before this)
            hip.stream_wait(self.stream, cur)
            blocks, self._deferred = self._deferred, []
            self._launch(blocks)
        self._forked = False
        hip.stream_wait(cur, self.stream)
