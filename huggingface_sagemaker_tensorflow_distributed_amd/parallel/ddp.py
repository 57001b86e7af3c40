"""Bucketed gradient all-reduce overlapped with backward (the ``hvd.DistributedOptimizer`` engine).

Reference: ``hvd.DistributedOptimizer(optimizer)`` (``scripts/train.py:114``) averages every
gradient across ranks through Horovod's background thread — per-step readiness negotiation with
rank 0, 64 MiB fusion buffer, ``ncclAllReduce``.

MI355X design:

* no negotiation: every rank's backward order is identical, so buckets are planned statically as
  contiguous slices of the flat gradient buffer (:class:`FlatParamStore`), in backward order;
* a bucket is launched (``all_reduce(SUM, async)`` on RCCL) the moment its last parameter gradient
  is written — gradients are written by the backward kernels straight into ``main_grad`` — so RCCL
  traffic runs on RCCL's own HIP stream underneath the rest of backward;
* the ``1/N`` average is folded into the optimizer kernel (no extra pass);
* on GPUs the bucket bookkeeping and the ``ncclAllReduce`` launches live in the native C++
  :class:`CommEngine` (``csrc/comm/comm_engine.cpp``: dedicated high-priority HIP stream, event
  ordering, no host sync); CPU/gloo worlds (tests) use ``torch.distributed`` with the same buckets;
* bucket size default is sized for xGMI: large enough that ring latency
  (≈tens of µs per collective) is amortised over 7 links, small enough that the tail bucket after
  the last backward kernel is short.
"""
from __future__ import annotations

import contextlib
import logging
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from . import backend
from .flat_params import FlatParamStore

logger = logging.getLogger(__name__)

DEFAULT_BUCKET_MB = float(os.environ.get("HSD_BUCKET_MB", "64"))
# wire compression of fp32 gradient buckets: name -> (CommEngine mode, torch dtype on the wire)
COMPRESSION = {"none": (0, None), "bf16": (1, torch.bfloat16), "fp16": (2, torch.float16)}

# Gradient wire format policy (``--grad_compression auto``, the default). bf16 on the wire halves the all-reduce bytes
# (bert-base 418 -> 209 MiB, bert-large 1,278 -> 639 MiB per step) at the price of two fused casts
# (fp32 -> bf16 before the all-reduce, back after it). Both the casts and the transfer run on the comm stream
# (csrc/comm/comm_engine.cpp launch_wire_cast, then ncclAllReduce), so the casts are weighed against the transfer time
# they save -- not against the backward they overlap with:
#
#   casts       CAST_S_PER_PARAM = 2.28e-12 s per parameter and step, measured on one MI355X (tools/wire_cast_cost.py,
#               profiles/wire_cast_r5.jsonl: 0.247 ms for bert-base's 109.5M gradients, 0.764 ms for bert-large's 335M)
#   transfer    a ring all-reduce moves 2(N-1)/N x S bytes per rank over the xGMI links RCCL's rings
#               can use: min(N-1, 7) point-to-point links of LINK_BPS = 153 GB/s (1 link at N = 2, 3 at N = 4, 7 at N = 8)
#   saved       2(N-1)/N x 2 bytes per parameter / (links x LINK_BPS): 13.1 ps at N = 2, 6.5 ps at N = 4, 3.3 ps at N = 8
#
# So bf16 wins at every N >= 2 whatever the step size, including the reference's own bert-large B = 8 S = 512 (N = 8:
# 1.10 ms of transfer saved for 0.76 ms of casts; N = 2: 4.4 ms saved), where the round-5 rule (casts vs 16 % of the
# backward) picked fp32. ``auto`` = bf16 for bf16 / fp8 runs on GPUs at N >= 2 when the model says it saves time, and
# fp32 on the wire for ``--dtype fp32`` -- the reference's precision and Horovod's uncompressed fp32 all-reduce
# (scripts/train.py:114; docs/PARITY.md 'gradient wire format'). Explicit ``none`` / ``bf16`` / ``fp16`` are kept.
CAST_S_PER_PARAM = 2.28e-12
LINK_BPS = 153e9
MAX_XGMI_LINKS = 7


def wire_times(world: int, n_params: int = 1) -> dict:
    """Comm-stream seconds for ``n_params`` fp32 gradients at ``world`` ranks: fp32 wire vs bf16 wire (+ casts)."""
    links = max(1, min(world - 1, MAX_XGMI_LINKS))
    ring = 2.0 * (world - 1) / world / (links * LINK_BPS)  # seconds per byte of payload per rank
    fp32 = 4 * n_params * ring
    bf16 = 2 * n_params * ring + CAST_S_PER_PARAM * n_params
    return {"links": links, "fp32_s": fp32, "bf16_s": bf16, "saved_s": fp32 - bf16}


def resolve_compression(requested: str, world: int, on_gpu: bool, dtype: str = "bf16") -> str:
    """The gradient wire format of a data-parallel job: ``requested`` unless it is ``auto`` (see the model above).
    ``dtype``: the run's compute dtype (``fp32`` keeps fp32 on the wire, the reference's numerics)."""
    if requested != "auto":
        return requested
    if world <= 1 or not on_gpu or dtype == "fp32":
        return "none"
    return "bf16" if wire_times(world)["saved_s"] > 0 else "none"


def overlap_from_timeline(backward_ms: float, buckets) -> dict:
    """``buckets``: (start_ms, end_ms, bytes) per bucket, all relative to the step's begin."""
    comm = sum(max(0.0, e - s) for s, e, _ in buckets)
    exposed = sum(max(0.0, e - max(s, backward_ms)) for s, e, _ in buckets)
    last = max((e for _, e, _ in buckets), default=backward_ms)
    nbytes = sum(b for _, _, b in buckets)
    return {"backward_ms": round(backward_ms, 4), "comm_ms": round(comm, 4), "exposed_ms": round(exposed, 4),
            "overlap_pct": round(100.0 * (1.0 - exposed / comm), 2) if comm > 0 else 100.0,
            "tail_ms": round(max(0.0, last - backward_ms), 4), "bytes": int(nbytes),
            "algbw_GBps": round(nbytes / (comm * 1e6), 2) if comm > 0 else None,
            "buckets": [[round(s, 4), round(e, 4), int(b)] for s, e, b in buckets]}


class _Bucket:
    __slots__ = ("index", "start", "end", "params", "ready", "handle", "launched", "wire")

    def __init__(self, index: int, start: int, end: int, params: List[int]):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.ready = set()
        self.handle = None
        self.launched = False
        self.wire = None


class GradBucketer:
    """Static buckets over a :class:`FlatParamStore`'s gradient buffer."""

    def __init__(self, store: FlatParamStore, bucket_mb: Optional[float] = None, group=None,
                 overlap: bool = True, native: Optional[bool] = None, engine=None, compression: str = "none"):
        """``engine``: an explicit native CommEngine (tests drive a world-of-one RCCL communicator through
        the full HIP backward with it; overlap is then on regardless of the world size).
        ``compression``: ``none`` | ``bf16`` | ``fp16`` — the dtype fp32 gradient buckets travel in
        (Horovod's ``hvd.Compression.fp16``): half the all-reduce bytes, gradients stay fp32 on either side."""
        if compression not in COMPRESSION:
            raise ValueError(f"compression {compression!r}: one of {sorted(COMPRESSION)}")
        self.compression = compression
        self.store = store
        self.group = group
        self.world = engine.world if engine is not None else backend.size()
        self.overlap = overlap and (self.world > 1 or engine is not None)
        self.bucket_bytes = int((bucket_mb or DEFAULT_BUCKET_MB) * (1 << 20))
        esize = store.grad.element_size()
        self.buckets: List[_Bucket] = []
        cur: List[int] = []
        start = 0
        for i, seg in enumerate(store.segments):
            cur.append(i)
            end = store.segments[i + 1].offset if i + 1 < len(store.segments) else store.numel
            if (end - start) * esize >= self.bucket_bytes or i + 1 == len(store.segments):
                self.buckets.append(_Bucket(len(self.buckets), start, end, cur))
                cur, start = [], end
        self._param_bucket = {}
        for b in self.buckets:
            for pi in b.params:
                self._param_bucket[pi] = b
        self.sync_enabled = True
        self._on_reduced = None
        self.last_launched: Optional[int] = None  # index of the last bucket whose all-reduce was issued (watchdog)
        self._prescale = 1.0
        self._hip = None
        self._capture_deps_pending = False
        self.engine = engine
        if engine is None and (native is None or native) and group is None:
            from .comm import get_engine

            try:
                self.engine = get_engine()
            except Exception as e:  # pragma: no cover - depends on the RCCL install
                logger.warning("native CommEngine unavailable (%s); using torch.distributed buckets", e)
                self.engine = None
        if self.engine is not None:
            if store.device.type == "cuda":
                from ..ops import hip as _hip

                side = _hip.side_stream(store.device)
                if side is not None:
                    self.engine.add_dependency_stream(side.cuda_stream)
                    self._hip = _hip
            param_bucket = [0] * len(store.segments)
            for b in self.buckets:
                for pi in b.params:
                    param_bucket[pi] = b.index
            self.engine.set_buckets(store.grad, [b.start for b in self.buckets], [b.end for b in self.buckets],
                                    [len(b.params) for b in self.buckets], param_bucket)
            if compression != "none" and store.grad.dtype == torch.float32:
                self.engine.set_compression(COMPRESSION[compression][0])
        store.ready_callback = self.mark_ready

    # ---------------------------------------------------------------- hooks
    def mark_ready(self, i: int) -> None:
        # no_sync micro-steps only accumulate: readiness is counted on the synced (last) micro-step alone,
        # on both paths, so a bucket fires once, after its gradients hold every micro-step's contribution
        if not self.sync_enabled:
            return
        if self.engine is not None:
            if self.overlap:
                if self._capture_deps_pending and self._hip.side_stream_in_capture():
                    # a whole-step graph capture (train/graph.py) has forked the wgrad side stream: from here on every
                    # bucket waits on that branch too, as in eager steps (the branch writes this bucket's main_grad)
                    self.engine.set_capture_deps(True)
                    self._capture_deps_pending = False
                idx = self.engine.mark_ready(i)
                if idx >= 0:
                    self.last_launched = idx
                    if self._on_reduced is not None:
                        self._on_reduced(idx)
            return
        b = self._param_bucket[i]
        if b.launched:
            raise RuntimeError(f"gradient for {self.store.names[i]} arrived after its bucket was reduced "
                               "(tied parameter used after its bucket completed?)")
        b.ready.add(i)
        if self.overlap and len(b.ready) == len(b.params):
            self._launch(b)

    def _launch(self, b: _Bucket) -> None:
        view = self.store.grad[b.start:b.end]
        if view.is_cuda:
            from ..ops import hip as _hip

            _hip.join_side_streams()  # gradients of this bucket may come from the wgrad stream
        wire_dtype = COMPRESSION[self.compression][1]
        if wire_dtype is not None and view.dtype == torch.float32:
            # fp16: pre-scaled by 1/micro-steps (the accumulated micro-step sum back to one step's magnitude, undone
            # in finish); the 1/world average stays in fp32 (optimizer grad_scale), as Horovod's fp16 compression
            # sums first and averages after: a 1/world pre-scale would push small gradients log2(world) binades
            # closer to fp16's subnormal range. bf16 has fp32's range and travels unscaled
            b.wire = (view * self._prescale).to(wire_dtype) if self._prescale != 1.0 else view.to(wire_dtype)
            b.handle = dist.all_reduce(b.wire, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            b.wire = None
            b.handle = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        b.launched = True
        self.last_launched = b.index

    # ---------------------------------------------------------------- step API
    def begin(self, micro_steps: int = 1) -> None:
        self.last_launched = None
        self._prescale = 1.0 / max(1, int(micro_steps)) if self.compression == "fp16" else 1.0
        if self.engine is not None:
            if self.compression == "fp16":
                self.engine.set_prescale(self._prescale)
            # inside a capture the engine waits on the wgrad branch only once the capture has forked it (mark_ready)
            self._capture_deps_pending = self._hip is not None
            self.engine.begin_step()
            return
        for b in self.buckets:
            b.ready.clear()
            b.handle = None
            b.launched = False

    def finish(self) -> None:
        """Launch any bucket not yet launched (unused params / no-overlap mode), then wait all."""
        if not self.sync_enabled:
            return
        if self.engine is not None:
            if self._hip is not None and self._hip.side_stream_in_capture():
                # a capture's last buckets: join the wgrad branch into the capture stream once, and order them after
                # the capture stream only -- an event recorded on the side stream after its final join would leave a
                # trailing node on a forked stream that no edge joins back
                self._hip.join_side_streams()
                self.engine.set_capture_deps(False)
            self.engine.finish()  # launches unlaunched buckets; compute stream waits (host does not)
            if self._on_reduced is not None:
                self.engine.wait_all()  # ... and for the optimizer slices queued behind the all-reduces
            return
        if self.world <= 1:
            return
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        for b in self.buckets:
            if b.handle is not None:
                b.handle.wait()
                b.handle = None
                if b.wire is not None:
                    g = self.store.grad[b.start:b.end]
                    g.copy_(b.wire)
                    if self._prescale != 1.0:
                        g.mul_(1.0 / self._prescale)
                    b.wire = None

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient-accumulation micro-steps: accumulate locally, no collective."""
        prev = self.sync_enabled
        self.sync_enabled = False
        try:
            yield
        finally:
            self.sync_enabled = prev

    def attach_optimizer(self, opt) -> bool:
        """Step each bucket's slice of ``opt`` (FusedAdam) on the RCCL engine's stream right after the bucket's
        all-reduce, i.e. under the rest of backward (native engine with overlap only)."""
        if self.engine is None or not self.overlap or self.store.device.type != "cuda":
            return False
        ext = torch.cuda.ExternalStream(self.engine.stream_ptr(), device=self.store.device)
        opt.enable_overlap([(b.start, b.end) for b in self.buckets])

        def on_reduced(idx: int) -> None:
            with torch.cuda.stream(ext):
                opt.step_range(idx)

        self._on_reduced = on_reduced
        return True

    # ---------------------------------------------------------------- overlap timeline
    def set_timing(self, on: bool) -> bool:
        """Record per-bucket HIP timing events from the next step on (native engine only)."""
        if self.engine is None:
            return False
        self.engine.set_timing(bool(on))
        return True

    def overlap_report(self) -> Optional[dict]:
        """Comm/compute overlap of the last step run with timing on (SURVEY.md §5 'comm-engine timestamps').

        ``backward_ms``: begin_step -> all backward kernels done (compute stream). Per bucket: start/end of its
        all-reduce on the comm stream. ``exposed_ms``: collective time after backward finished, i.e. what the
        step pays on top of compute; ``overlap_pct`` = 100 * (1 - exposed / total collective time)."""
        if self.engine is None:
            return None
        t = list(self.engine.timings())
        if not t:
            return None
        return overlap_from_timeline(t[0], [tuple(t[i:i + 3]) for i in range(1, len(t), 3)])

    def detach(self) -> None:
        self.store.ready_callback = None
