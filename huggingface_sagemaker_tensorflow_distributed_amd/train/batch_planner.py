"""Per-GPU batch sizing for the HBM of the device (``--train_batch_size auto``).

The reference hard-codes ``train_batch_size=8`` for a 16-GB V100 (``launch.py:15``). An MI355X has 288 GB of HBM3E,
so the useful per-GPU batch is set by memory and by where throughput stops growing, not by a fixed number. This
planner measures instead of guessing:

1. After the weights, the flat fp32 master / bf16 compute / gradient buffers and the optimizer state exist, it runs
   one forward + backward at two probe batches (no optimizer step, gradients zeroed afterwards, no collective:
   the store's readiness callback is not attached yet) and reads the allocator's peak for each.
2. Peak memory is linear in the batch (activations kept for the backward + the backward's transient buffers), so
   the two probes give ``peak(B) = fixed + per_seq * B``.
3. The budget is ``headroom * total HBM`` minus what other processes / runtimes already hold on the device; the
   batch is the largest multiple of ``multiple`` under it, capped at ``max_tokens / seq_len`` (the throughput
   knee: bert-base S = 128 runs 11.9k seq/s at B = 1024 and 12.0k at B = 2048, README 'Measured'), and agreed
   across data-parallel ranks (minimum).

Without a GPU the same formula runs on an analytic activation estimate (:func:`activation_bytes_per_seq`) against
``fallback_budget_bytes``. With ``--dtype fp8`` the probes' forward passes also record the first amax values of the
delayed-scaling sites (a random batch of the training shape), as a warm-up step would.
"""
from __future__ import annotations

import logging
from dataclasses import asdict, dataclass
from typing import Optional

import torch

logger = logging.getLogger(__name__)

DEFAULT_MAX_TOKENS = 131072  # bert-base S=128 B=1024: the measured throughput knee on one MI355X


@dataclass
class BatchPlan:
    per_gpu_batch: int
    seq_len: int
    per_seq_bytes: float
    fixed_bytes: float
    budget_bytes: float
    total_bytes: float
    method: str  # "probe" (measured on the device) or "analytic"
    capped_by: str  # "memory" | "max_tokens" | "min"
    predicted_peak_bytes: float

    def as_dict(self) -> dict:
        return asdict(self)


def activation_bytes_per_seq(cfg, seq_len: int, act_bytes: int = 2) -> float:
    """Bytes one sequence keeps alive from forward to backward on the HIP path, plus the backward's largest
    transient, per encoder layer x layers. Per token and layer the forward keeps: QKV (3H), attention output (H),
    the out-projection result and its LayerNorm (2H), FFN1's GELU and GELU' (2I), FFN2's result and LayerNorm
    (2H), one fp32 LSE per head and two fp32 LN statistics per LayerNorm; the backward's transients peak at the
    FFN (a [T, I] gradient plus a [T, 3H] attention gradient)."""
    H, I, L, heads = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers, cfg.num_attention_heads
    kept = (3 * H + H + 2 * H + 2 * I + 2 * H) * act_bytes + heads * 4 + 2 * 2 * 4
    transient = (I + 3 * H) * act_bytes
    embed = 2 * H * act_bytes
    return float(seq_len * (L * kept + transient + embed))


def _round_down(x: float, multiple: int) -> int:
    return max(0, int(x) // multiple * multiple)


def choose(per_seq: float, fixed: float, budget: float, seq_len: int, *, multiple: int = 8,
           max_tokens: Optional[int] = DEFAULT_MAX_TOKENS, min_batch: int = 1):
    """(batch, capped_by) for the linear memory model ``fixed + per_seq * B <= budget``."""
    if per_seq <= 0:
        raise ValueError("per-sequence bytes must be positive")
    b_mem = _round_down((budget - fixed) / per_seq, multiple)
    capped_by = "memory"
    b = b_mem
    if max_tokens:
        b_tok = _round_down(max_tokens / seq_len, multiple) or max(1, max_tokens // seq_len)
        if b_tok < b:
            b, capped_by = b_tok, "max_tokens"
    if b < min_batch:
        b, capped_by = min_batch, "min"
    return b, capped_by


def _probe_peak(model, store, cfg, batch: int, seq_len: int, device) -> int:
    g = torch.Generator(device="cpu").manual_seed(1234 + batch)
    ids = torch.randint(1000, cfg.vocab_size, (batch, seq_len), generator=g).to(device)
    am = torch.ones(batch, seq_len, dtype=torch.long, device=device)
    labels = torch.randint(0, max(2, cfg.num_labels), (batch,), generator=g).to(device)
    if model.__class__.__name__ == "RobertaForMaskedLM":
        labels = torch.full((batch, seq_len), -100, dtype=torch.long, device=device)
        labels[:, ::7] = ids[:, ::7]
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(device)
    was_training = model.training
    model.train()
    model.rng.new_step(0)
    loss, _ = model(ids, attention_mask=am, labels=labels)
    loss.backward()
    torch.cuda.synchronize(device)
    peak = torch.cuda.max_memory_allocated(device)
    del loss, ids, am, labels
    store.zero_grad()
    from .. import ops

    ops.join_side_streams()
    model.train(was_training)
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()
    return peak


def _shadow_bytes(store, compression: str) -> float:
    if compression in (None, "none") or store.grad.dtype != torch.float32:
        return 0.0
    return float(store.numel) * 2


def plan(model, store, seq_len: int, device, *, headroom: float = 0.9, multiple: int = 8,
         max_tokens: Optional[int] = DEFAULT_MAX_TOKENS, probe_batches=None,
         fallback_budget_bytes: float = 64 * 2**30, compression: str = "none") -> BatchPlan:
    """Largest per-GPU batch whose training step fits ``headroom`` of the device memory (see module doc).

    The two probes run with the weight-gradient side stream OFF (the large-batch regime the chosen batch usually
    lands in); when the chosen batch is small enough for the side stream to be on, its peak is re-measured in that
    regime and the batch shrunk if the stash of wgrad operands pushes it over budget. ``compression`` != ``none``
    adds the data-parallel engine's 16-bit shadow of the gradient buffer (created after planning) to the fixed
    bytes."""
    cfg = model.cfg
    device = torch.device(device)
    if device.type == "cuda":
        from ..ops import hip as _hip

        # probes of >= 8192 tokens run the large-batch kernel paths (no small-grid split-K workspaces)
        b1, b2 = probe_batches or (max(8, 8192 // seq_len), 2 * max(8, 8192 // seq_len))
        with _hip.wgrad_stream_override("0"):
            p1 = _probe_peak(model, store, cfg, b1, seq_len, device)
            p2 = _probe_peak(model, store, cfg, b2, seq_len, device)
        per_seq = max(1.0, (p2 - p1) / float(b2 - b1))
        fixed = p1 - per_seq * b1 + _shadow_bytes(store, compression)
        free, total = torch.cuda.mem_get_info(device)
        others = max(0, total - free - torch.cuda.memory_reserved(device))  # other processes / runtime pools
        budget = headroom * total - others
        method = "probe"
        b, capped_by = choose(per_seq, fixed, budget, seq_len, multiple=multiple, max_tokens=max_tokens)
        if b > 0 and _hip.wgrad_side_stream_for(b * seq_len):
            peak = _probe_peak(model, store, cfg, b, seq_len, device) + _shadow_bytes(store, compression)
            method = "probe+side-stream"
            if peak > budget:
                # the side-stream stash adds a per-sequence term: rescale the slope to the measured peak
                per_seq = max(per_seq, (peak - fixed) / float(b))
                b, capped_by = choose(per_seq, fixed, budget, seq_len, multiple=multiple, max_tokens=max_tokens)
        return BatchPlan(per_gpu_batch=b, seq_len=seq_len, per_seq_bytes=per_seq, fixed_bytes=fixed,
                         budget_bytes=budget, total_bytes=float(total), method=method, capped_by=capped_by,
                         predicted_peak_bytes=fixed + per_seq * b)
    else:
        per_seq = activation_bytes_per_seq(cfg, seq_len, 4 if store.compute_dtype == torch.float32 else 2)
        fixed = float(store.numel) * (4 * 4 + store.compute.element_size())  # master, grad, m, v, compute copy
        fixed += _shadow_bytes(store, compression)
        total = float(fallback_budget_bytes)
        budget = headroom * total
        method = "analytic"
    b, capped_by = choose(per_seq, fixed, budget, seq_len, multiple=multiple, max_tokens=max_tokens)
    return BatchPlan(per_gpu_batch=b, seq_len=seq_len, per_seq_bytes=per_seq, fixed_bytes=fixed,
                     budget_bytes=budget, total_bytes=float(total), method=method, capped_by=capped_by,
                     predicted_peak_bytes=fixed + per_seq * b)


def agree_min(batch: int, device) -> int:
    """Every data-parallel rank runs the same per-GPU batch: the minimum of the ranks' plans."""
    from ..parallel import backend

    if not backend.is_distributed():
        return batch
    t = torch.tensor([batch], dtype=torch.int64, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
    return int(t.item())
