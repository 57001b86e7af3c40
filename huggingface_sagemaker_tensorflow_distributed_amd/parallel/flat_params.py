"""Flat parameter / gradient / optimizer-state storage.

MI355X-first memory layout: every parameter of the model lives inside ONE flat fp32 master buffer,
ONE flat compute-dtype (bf16) buffer whose views the kernels read, and ONE flat gradient buffer
(``main_grad`` views) that the backward kernels write directly (no per-parameter allocation, no
``AccumulateGrad`` pass, no bucket pack copy: a gradient bucket is a contiguous slice). The
optimizer is then a single launch over flat buffers, and broadcast/all-reduce are single
collectives over slices — the replacement for Horovod's 64 MiB fusion buffer.

Layout order is *reverse* declaration order (== approximately backward order), so gradient buckets
complete front-to-back while backward is still running.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn as nn

ALIGN = 64  # elements; keeps every view 128-B (bf16) / 256-B (fp32) aligned for 16-B vector IO

# 2-D weights whose transposed bf16 copy the dgrad GEMMs read (B operand of dX = dY·W is Wᵀ, k-contiguous)
TRANSPOSED_WEIGHTS = re.compile(r"(^|\.)layers\.\d+\.(qkv|attn_out|ffn1|ffn2)_weight$")


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


@dataclass
class Segment:
    name: str
    offset: int
    numel: int
    shape: tuple
    decay: bool


def _no_decay(name: str) -> bool:
    leaf = name.rsplit(".", 1)[-1]
    toks = leaf.split("_")
    return leaf.endswith("bias") or any(t in ("ln", "ln1", "ln2") for t in toks)


# Below this many tokens per rank the dgrad GEMMs read W directly (gemm2 NT with a k-strided B operand) instead of a
# stored Wᵀ copy: the per-step Wᵀ refresh (2 x the encoder's bf16 weights through HBM) is a fixed cost that small
# steps cannot amortise (3 % of the reference's own bert-large B = 8 S = 512 step), while at large token counts the
# k-contiguous B read is the cheaper main loop. HSD_WT: auto (default) | 1 (always keep Wᵀ) | 0 (never).
WT_MIN_TOKENS = int(os.environ.get("HSD_WT_MIN_TOKENS", "32768"))


def keep_transposed_weights(rank_tokens) -> bool:
    mode = os.environ.get("HSD_WT", "auto").lower()
    if mode in ("0", "1"):
        return mode == "1"
    return rank_tokens is None or rank_tokens >= WT_MIN_TOKENS


def hip_kernels_active() -> bool:
    return os.environ.get("HSD_OPS", "").lower() != "torch"


class FlatParamStore:
    def __init__(self, model: nn.Module, device: torch.device, compute_dtype: torch.dtype = torch.float32,
                 grad_dtype: torch.dtype = torch.float32, fp8: bool = False, transposed: bool = True):
        """``transposed``: keep bf16 Wᵀ copies of the encoder weights for the dgrad GEMMs (refreshed after every
        optimizer step); False = the dgrads read W directly (small steps, see keep_transposed_weights). fp8 always
        keeps them (the fp8 dgrad reads the quantised Wᵀ)."""
        self.device = torch.device(device)
        self.fp8 = fp8
        self.keep_wt = bool(transposed) or fp8
        self.compute_dtype = compute_dtype
        self.grad_dtype = grad_dtype
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        named = list(reversed(named))
        self.params: List[nn.Parameter] = [p for _, p in named]
        self.names: List[str] = [n for n, _ in named]
        self.segments: List[Segment] = []
        off = 0
        for n, p in named:
            self.segments.append(Segment(n, off, p.numel(), tuple(p.shape), not _no_decay(n)))
            off = _round_up(off + p.numel(), ALIGN)
        self.numel = _round_up(off, 1024)
        # ---- buffers
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for seg, p in zip(self.segments, self.params):
                self.master[seg.offset:seg.offset + seg.numel].copy_(p.detach().reshape(-1).to(torch.float32))
        if compute_dtype == torch.float32:
            self.compute = self.master
        else:
            self.compute = self.master.to(compute_dtype)
        self.grad = torch.zeros(self.numel, dtype=grad_dtype, device=self.device)
        # decay mask per 64-element block (optimizer segment table)
        for seg, p in zip(self.segments, self.params):
            p.data = self.compute[seg.offset:seg.offset + seg.numel].view(seg.shape)
            p.main_grad = self.grad[seg.offset:seg.offset + seg.numel].view(seg.shape)
            p.grad = None
        self._index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        self._setup_transposed()
        self._setup_splits()
        # gradient-ready notification: HIP backward kernels write main_grad directly and return None;
        # torch-autograd gradients (CPU path, small torch-op heads) are folded into main_grad here. Either
        # way autograd runs the post-accumulate hook exactly once per parameter per backward, after every
        # node that used it (tied weights included), and that hook is the ONE readiness signal.
        self.ready_callback = None
        self._hooks = []
        for i, p in enumerate(self.params):
            p._hsd_ready = self._make_ready(i)
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_accum_hook(i)))

    def _make_ready(self, i: int):
        def ready():
            cb = self.ready_callback
            if cb is not None:
                cb(i)
        return ready

    # The post-accumulate hook below is also where the overlapped optimizer (optim/adam.py enable_overlap) may
    # start updating this parameter: see the invariant documented there.
    def _make_accum_hook(self, i: int):
        def hook(p):
            if p.grad is not None:
                p.main_grad.add_(p.grad.to(p.main_grad.dtype))
                p.grad = None
            p._hsd_ready()
        return hook

    # ----------------------------------------------------------------------------------
    def _setup_splits(self) -> None:
        """fp32 compute on the GPU (the reference's precision, ops/hip32.py): bf16 hi / lo halves of every parameter
        (hi = bf16(θ), lo = bf16(θ - hi)) for the split-product GEMMs, written by the fused Adam in the same pass as
        the update -- the weights are split once per optimizer step, not at every forward / backward use."""
        self.split_hi = self.split_lo = None
        self._split_version = None
        if self.device.type != "cuda" or self.compute_dtype != torch.float32 or not hip_kernels_active():
            return
        self.split_hi = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
        self.split_lo = torch.empty_like(self.split_hi)
        for seg, p in zip(self.segments, self.params):
            p._hsd_split = [self.split_hi[seg.offset:seg.offset + seg.numel].view(seg.shape),
                            self.split_lo[seg.offset:seg.offset + seg.numel].view(seg.shape), self, p._version]
        self.refresh_splits()

    @torch.no_grad()
    def refresh_splits(self) -> None:
        """Re-split every parameter (after anything other than the optimizer step changed the weights) and record the
        versions the halves are current for (ops/hip32.py weight_split re-splits a weight changed in place since)."""
        if self.split_hi is None:
            return
        from ..ops import hip

        hip._C.split2(self.master, self.split_hi, self.split_lo)
        self._split_version = self.master._version
        for p in self.params:
            p._hsd_split[3] = p._version

    def splits_current(self) -> bool:
        return self._split_version is not None and self.master._version == self._split_version

    def adam_outputs(self, start: int, end: int):
        """(out, out_lo) for the fused Adam on flat slice [start, end): the bf16 compute copy (bf16 / fp8 runs), or the
        fp32 run's hi / lo halves, or (None, None)."""
        if self.split_hi is not None:
            return self.split_hi[start:end], self.split_lo[start:end]
        if self.compute is not self.master:
            return self.compute[start:end], None
        return None, None

    def _setup_transposed(self) -> None:
        """bf16 Wᵀ copies (one flat buffer) for the dgrad GEMMs, refreshed by ONE batched transpose launch
        after every optimizer step instead of a transpose per GEMM per step."""
        self.transposed = None
        self._tdesc = None
        self._fp8_desc = None
        if self.device.type != "cuda" or self.compute_dtype != torch.bfloat16 or not self.keep_wt:
            return
        idx = [i for i, n in enumerate(self.names) if TRANSPOSED_WEIGHTS.search(n) and len(self.segments[i].shape) == 2
               and self.segments[i].shape[0] % 4 == 0 and self.segments[i].shape[1] % 4 == 0]
        if not idx:
            return
        total = sum(self.segments[i].numel for i in idx)
        self.transposed = torch.empty(total, dtype=self.compute_dtype, device=self.device)
        desc, off, tiles = [], 0, 0
        for i in idx:
            rows, cols = self.segments[i].shape
            p = self.params[i]
            wt = self.transposed[off:off + rows * cols].view(cols, rows)
            p._hsd_wt = wt
            desc.append([p.data.data_ptr(), wt.data_ptr(), rows, cols, tiles])
            tiles += ((rows + 63) // 64) * ((cols + 63) // 64)
            off += rows * cols
        self._tdesc = torch.tensor(desc, dtype=torch.int64, device=self.device)
        self._ttiles = tiles
        self._fp8_desc = None
        if self.fp8:
            self._setup_fp8(idx)
        self.refresh_transposed()

    def _setup_fp8(self, idx) -> None:
        """fp8 (e4m3) copies of every encoder weight W and of its stored transpose Wᵀ, with one per-tensor
        scale shared by both: the forward GEMM reads W8, the dgrad GEMM W8ᵀ. All
        of them are re-quantised by two batched launches (amax, quantise) after every optimizer step."""
        from ..ops import hip

        import os

        per_block = hip._C.fp8_elems_per_block()
        total = sum(self.segments[i].numel for i in idx)
        self.fp8_w = torch.empty(total, dtype=torch.uint8, device=self.device)
        self.fp8_wt = torch.empty(total, dtype=torch.uint8, device=self.device)
        # one 128-B line per weight for its amax / scale: every block of the amax pass ends with an atomic on its
        # weight's slot, and packed slots put all ~18k of them on one L2 line (roberta-large: 514 us for a 604 MB
        # read, 1.2 TB/s; profiles/fp8_refresh_r5.log): 32 floats per slot.
        slot = 32
        self.fp8_amax = torch.zeros(len(idx) * slot, dtype=torch.float32, device=self.device)
        self.fp8_sinv = torch.ones(len(idx) * slot, dtype=torch.float32, device=self.device)
        # delayed-scaling history of the two activation-side quantisation sites of each weight:
        # [weight][0 = forward input x, 1 = dgrad input dy][0 = amax used for this step's scale, 1 = running]
        self.fp8_act = torch.zeros(len(idx), 2, 2, dtype=torch.float32, device=self.device)
        amax_rows, quant_rows, ab, qb, off = [], [], 0, 0, 0
        for t, i in enumerate(idx):
            rows, cols = self.segments[i].shape
            n = rows * cols
            p = self.params[i]
            q = self.fp8_w[off:off + n].view(rows, cols)
            qt = self.fp8_wt[off:off + n].view(cols, rows)
            p._hsd_q, p._hsd_qt, p._hsd_qs = q, qt, self.fp8_sinv[t * slot:t * slot + 1]
            p._hsd_fp8_x, p._hsd_fp8_g = self.fp8_act[t, 0], self.fp8_act[t, 1]
            nb = (n + per_block - 1) // per_block
            amax_rows.append([p.data.data_ptr(), 0, n, t * slot, ab])
            ab += nb
            quant_rows.append([p.data.data_ptr(), q.data_ptr(), n, t * slot, qb])
            qb += nb
            quant_rows.append([p._hsd_wt.data_ptr(), qt.data_ptr(), n, t * slot, qb])
            qb += nb
            off += n
        self._fp8_desc = (torch.tensor(amax_rows, dtype=torch.int64, device=self.device), ab,
                          torch.tensor(quant_rows, dtype=torch.int64, device=self.device), qb)

    @torch.no_grad()
    def refresh_fp8(self) -> None:
        if self._fp8_desc is None:
            return
        from ..ops import hip

        ad, ab, qd, qb = self._fp8_desc
        self._roll_fp8_act()
        self.fp8_amax.zero_()
        hip._C.fp8_quant_many(ad, ab, qd, qb, self.fp8_amax, self.fp8_sinv, 0)
        # the slots are left zero (stream-ordered after the quantise pass read them): per-slice passes
        # (refresh_fp8_subset) accumulate into them next
        self.fp8_amax.zero_()

    def _roll_fp8_act(self) -> None:
        # roll the activation amax history: next step scales with this step's amax (sites not used this
        # step keep their previous value)
        prev, cur = self.fp8_act[..., 0], self.fp8_act[..., 1]
        prev.copy_(torch.where(cur > 0, cur, prev))
        cur.zero_()

    def fp8_subsets(self, ranges) -> list:
        """Per flat-buffer slice ``[start, end)``: the fp8 amax / quantise descriptor tables of the fp8 weights inside
        it (or ``None``), so an optimizer that steps slices separately re-quantises each slice's weights (W8 and W8ᵀ,
        after the slice's Wᵀ refresh) right after its update, under the backward, instead of in one pass over every
        weight at the end of the step (:meth:`refresh_fp8_subset`, :meth:`finish_fp8_step`)."""
        if self._fp8_desc is None:
            return [None] * len(ranges)
        from ..ops import hip

        per_block = hip._C.fp8_elems_per_block()
        ad, _ab, qd, _qb = self._fp8_desc
        arows, qrows = ad.cpu().tolist(), qd.cpu().tolist()
        base = self.compute.data_ptr()
        esize = self.compute.element_size()
        out = []
        for st, e in ranges:
            a_sub, q_sub, ab, qb = [], [], 0, 0
            for t, (src, dst, n, slot, _b) in enumerate(arows):
                off = (src - base) // esize
                if not (st <= off < e):
                    continue
                nb = (n + per_block - 1) // per_block
                a_sub.append([src, dst, n, slot, ab])
                ab += nb
                for qr in qrows[2 * t:2 * t + 2]:
                    q_sub.append([qr[0], qr[1], qr[2], qr[3], qb])
                    qb += nb
            if a_sub:
                out.append((torch.tensor(a_sub, dtype=torch.int64, device=self.device), ab,
                            torch.tensor(q_sub, dtype=torch.int64, device=self.device), qb))
            else:
                out.append(None)
        return out

    @torch.no_grad()
    def refresh_fp8_subset(self, sub) -> None:
        """Re-quantise one slice's fp8 weights (a :meth:`fp8_subsets` entry) on the current stream; their amax slots
        were zeroed by the previous :meth:`finish_fp8_step` (or the store's construction)."""
        if sub is None:
            return
        from ..ops import hip

        ad, ab, qd, qb = sub
        hip._C.fp8_quant_many(ad, ab, qd, qb, self.fp8_amax, self.fp8_sinv, 0)

    @torch.no_grad()
    def finish_fp8_step(self) -> None:
        """End of a step whose slices re-quantised their own fp8 weights: roll the activation amax history and zero
        the weight amax slots for the next step's per-slice passes."""
        if self._fp8_desc is None:
            return
        self._roll_fp8_act()
        self.fp8_amax.zero_()

    def transposed_subsets(self, ranges) -> list:
        """Per flat-buffer slice ``[start, end)``: the batched-transpose descriptor table of the weights inside it
        (``(desc, tiles)`` or ``None``), so an optimizer that steps slices separately can refresh each slice's Wᵀ
        right after the slice's update instead of in one pass at the end of the step."""
        if self._tdesc is None:
            return [None] * len(ranges)
        rows_all = self._tdesc.cpu().tolist()
        base = self.compute.data_ptr()
        esize = self.compute.element_size()
        out = []
        for st, e in ranges:
            desc, tiles = [], 0
            for src, dst, rows, cols, _t in rows_all:
                off = (src - base) // esize
                if st <= off < e:
                    desc.append([src, dst, rows, cols, tiles])
                    tiles += ((rows + 63) // 64) * ((cols + 63) // 64)
            out.append((torch.tensor(desc, dtype=torch.int64, device=self.device), tiles) if desc else None)
        return out

    @torch.no_grad()
    def refresh_transposed(self) -> None:
        if self._tdesc is None:
            return
        from ..ops import hip

        hip._C.transpose_many(self._tdesc, self._ttiles)
        self.refresh_fp8()

    @torch.no_grad()
    def refresh_transposed_subset(self, subset) -> None:
        """Wᵀ refresh of one slice (a :meth:`transposed_subsets` entry) on the current stream."""
        if subset is None:
            return
        from ..ops import hip

        hip._C.transpose_many(subset[0], subset[1])

    def index_of(self, p: torch.Tensor) -> int:
        return self._index[id(p)]

    def segment_of(self, p: torch.Tensor) -> Segment:
        return self.segments[self._index[id(p)]]

    def zero_grad(self) -> None:
        if self.grad.is_cuda and hip_kernels_active():
            from ..ops import hip

            hip._C.memset0(self.grad)  # hipMemsetAsync: no elementwise fill kernel in the step
        else:
            self.grad.zero_()

    @torch.no_grad()
    def sync_compute_from_master(self) -> None:
        if self.compute is not self.master:
            self.compute.copy_(self.master)
        self.refresh_transposed()
        self.refresh_splits()

    def decay_block_mask(self, block: int) -> torch.Tensor:
        """uint8 per ``block`` elements: 1 = apply weight decay. Segments are ALIGN-aligned."""
        assert block % ALIGN == 0 or ALIGN % block == 0
        nb = self.numel // block
        m = torch.zeros(nb, dtype=torch.uint8)
        for s in self.segments:
            if s.decay:
                m[s.offset // block: (s.offset + s.numel + block - 1) // block] = 1
        return m.to(self.device)

    def state_dict(self) -> dict:
        return {"master": self.master.detach().cpu(), "names": list(self.names),
                "offsets": [s.offset for s in self.segments]}

    @torch.no_grad()
    def load_master(self, master: torch.Tensor) -> None:
        self.master.copy_(master.to(self.device))
        self.sync_compute_from_master()
