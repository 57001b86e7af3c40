"""HIP (gfx950) implementations of the fused ops, as autograd Functions over ``_C`` kernels.

Parameter gradients never go through autograd's ``AccumulateGrad``: the backward kernels add them
(fp32) straight into the parameter's slice of the flat ``main_grad`` buffer
(:class:`parallel.FlatParamStore`) and return ``None`` for it. Readiness for the gradient bucket's RCCL
all-reduce is signalled once per parameter by the store's post-accumulate hook, which autograd runs
right after the last node that used the parameter (so a tied weight — MLM decoder = word embeddings —
is signalled only after both of its contributions). Without a store (unit tests) the gradient is
returned normally.
"""
from __future__ import annotations

from typing import Optional

import weakref

import torch

from ._ext import load

_C = load()


def _s64(seed: int) -> int:
    seed &= (1 << 64) - 1
    return seed - (1 << 64) if seed >= (1 << 63) else seed


class _Grad:
    """fp32 accumulation target for one parameter's gradient."""

    __slots__ = ("p", "mg", "buf")

    def __init__(self, p: torch.Tensor):
        self.p = p
        mg = getattr(p, "main_grad", None)
        self.mg = mg
        if mg is not None and mg.dtype == torch.float32:
            self.buf = mg
        else:
            self.buf = torch.zeros(p.shape, dtype=torch.float32, device=p.device)

    def done(self):
        if self.mg is None:
            return self.buf.to(self.p.dtype)
        if self.buf is not self.mg:
            self.mg.add_(self.buf.to(self.mg.dtype))
        return None  # bucket readiness: FlatParamStore's post-accumulate hook (fires once, after all uses)


# ------------------------------------------------------------------------------------------ wgrad stream
# Weight-gradient GEMMs are independent of the rest of the backward chain (dgrad -> previous layer), so
# they run on a side stream: their compute overlaps the dgrad GEMMs' memory-bound epilogues and the
# attention / LayerNorm kernels on other CUs. Gradient readiness (bucket all-reduce) is signalled from
# the side stream; the comm engine and the overlapped optimizer order their work after it, and every backward
# pass ends with the compute stream joined to it (an autograd final callback), so gradients read after
# ``loss.backward()`` are complete on the compute stream.
#
# HSD_WGRAD_STREAM: "auto" (default) = on for steps of <= 131,072 tokens. Small steps, where the GEMM grids leave CUs
# idle, measured +1.6 % (bert-base B = 256) to +8.4 % (bert-base B = 64) and +5.8 % at the reference's bert-large
# B = 8 S = 512 (profiles/wgrad_stream_small_ab_r2.log). At the headline's 131,072 tokens it was neutral while the
# persistent GEMMs walked static tile lists; with dynamic tile claims a persistent dgrad kernel shares the CUs with the
# one-shot weight-gradient grid and the side stream measured +0.7 % (13,385 vs 13,285 seq/s,
# profiles/wgrad_side_stream_b1024_ab_r4.log). Off above. "1" = always, "0" = never.
import os as _os

_WGRAD_MODE = _os.environ.get("HSD_WGRAD_STREAM", "auto").strip().lower()
_WGRAD_AUTO_MAX_TOKENS = int(_os.environ.get("HSD_WGRAD_STREAM_MAX_TOKENS", "131072"))
# The side stream's operands stay referenced until the next join_side_streams() instead of record_stream (the compute
# stream has then waited for the side stream, so their blocks go back to the compute stream's pool with no cross-stream
# event bookkeeping in the allocator; record_stream collapsed throughput 7x at B = 256-1024). Costs the operands' memory
# until the end of the backward. The fork is the extension's stream_wait + gemm2_on (no Python stream plumbing).
_SIDE = {}
_STASH = []
_JOIN_QUEUED = [False]
# callbacks run right after each weight-gradient fork (main -> side stream) outside captures, with the side stream:
# work that must follow everything queued on the compute stream so far can be ordered behind the side stream's
# position instead of recording an event of its own on the compute stream (optim/adam.py LocalOverlap: each event
# recorded on the compute stream costs ~3 us on it, tools/fork_cost.py)
_FORK_LISTENERS = []
# HIP-graph capture (train/graph.py): the capture stream the side stream forks from and joins back to (autograd's
# end-of-backward callback runs with the device's default stream current, not the capture stream), and whether this
# capture forked it.
_CAPTURE = {"parent": None, "forked": False}
# HSD_TEST_SIDE_DELAY_US: test-only stall queued on the side stream before each backward's first weight gradient
_SIDE_DELAY_US = float(_os.environ.get("HSD_TEST_SIDE_DELAY_US", "0"))


def begin_capture(parent) -> None:
    """Called by a graph capture before its forward: the wgrad side stream becomes a branch of the capture."""
    _CAPTURE["parent"], _CAPTURE["forked"] = parent, False


CAPTURES_WITH_SIDE_STREAM = [0]  # captures that branched the side stream (tests/test_gpu_graph.py)


def end_capture() -> None:
    if _CAPTURE["forked"]:
        CAPTURES_WITH_SIDE_STREAM[0] += 1
    _CAPTURE["parent"], _CAPTURE["forked"] = None, False


def side_stream_in_capture() -> bool:
    """Whether the running capture has forked the wgrad side stream (waits on it are then capture edges)."""
    return _CAPTURE["forked"]


def side_stream_waitable() -> bool:
    """Whether work may wait on the wgrad side stream now: always outside a capture; inside one only once the capture
    has forked it (an event of a stream outside the capture is no capture edge)."""
    return _CAPTURE["parent"] is None or _CAPTURE["forked"]


# Cross-stream ordering without a new event per call. ``Stream.wait_stream`` creates (and on ROCm lazily
# hipEventCreate's) a fresh event every time and goes through torch's Python stream plumbing; with ~80 forks / joins
# per step (weight-gradient side stream, optimizer slices) small-batch steps were host-bound
# (tools/cpu_profile_step.py). The extension records an event from a per-thread ring instead; a wait takes the
# event's state at the time of the call, so re-recording it later does not move an earlier wait.


def stream_wait(dst, src) -> None:
    """``dst`` waits for everything queued on ``src`` so far (``dst.wait_stream(src)`` with an event from the
    extension's per-thread ring). Streams or raw handles; ``None`` / 0 = the current stream."""
    _C.stream_wait(dst.cuda_stream if hasattr(dst, "cuda_stream") else int(dst or 0),
                   src.cuda_stream if hasattr(src, "cuda_stream") else int(src or 0))


def side_stream(device) -> Optional[torch.cuda.Stream]:
    """The device's wgrad side stream (created on first use), or None when HSD_WGRAD_STREAM=0."""
    if _WGRAD_MODE in ("0", "off", "false"):
        return None
    key = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(key)
    if s is None:
        # (a CU-masked side stream -- hipExtStreamCreateWithCUMask, half or 3/4 of the CUs, so the compute stream
        # always finds CUs free of weight-gradient workgroups -- measured 18-47 % slower:
        # profiles/r6/side_stream_cu_mask_rejected_r6.log)
        s = torch.cuda.Stream(device=key)
        _SIDE[key] = s
    return s


def _use_side_stream(tokens: int) -> bool:
    if _WGRAD_MODE in ("0", "off", "false"):
        return False
    if torch.cuda.is_current_stream_capturing() and _CAPTURE["parent"] is None:
        return False
    return _WGRAD_MODE in ("1", "on", "true") or tokens <= _WGRAD_AUTO_MAX_TOKENS


def wgrad_side_stream_for(tokens: int) -> bool:
    """Whether a step of ``tokens`` tokens runs its weight gradients on the side stream (the batch planner sizes
    the memory regime with it: the side stream's stash keeps the wgrad operands alive until the end of backward)."""
    return _use_side_stream(tokens)


class wgrad_stream_override:  # noqa: N801 - used as a context manager
    """Temporarily force HSD_WGRAD_STREAM (``"0"`` / ``"1"`` / ``"auto"``), e.g. for memory probes."""

    def __init__(self, mode: str):
        self.mode = mode

    def __enter__(self):
        global _WGRAD_MODE
        self.prev, _WGRAD_MODE = _WGRAD_MODE, self.mode
        return self

    def __exit__(self, *exc):
        global _WGRAD_MODE
        _WGRAD_MODE = self.prev
        return False


def join_side_streams() -> None:
    """Make the current stream wait for every side stream (call before consuming gradients). Inside a HIP graph
    capture the capture stream joins the side stream, if this capture forked it (else nothing to join)."""
    if not _SIDE:
        return
    parent = _CAPTURE["parent"]
    if parent is not None:
        if _CAPTURE["forked"]:
            for s in _SIDE.values():
                if s.device == parent.device:
                    _C.stream_wait(parent.cuda_stream, s.cuda_stream)
        _STASH.clear()
        _JOIN_QUEUED[0] = False
        return
    if torch.cuda.is_current_stream_capturing():
        return
    dev = torch.cuda.current_device()
    for k, s in _SIDE.items():
        if k == dev:
            _C.stream_wait(0, s.cuda_stream)
    _STASH.clear()
    _JOIN_QUEUED[0] = False


def _end_of_backward() -> None:
    join_side_streams()


def _launch_wgrad(s, g: "_Grad", dy, x, dyq, xq):
    """g += dyᵀ·x on the side stream ``s`` (already ordered after dy / x); the g.done() result."""
    N, K, T = dy.shape[1], x.shape[1], dy.shape[0]
    if g.buf is g.mg and _wgrad8_ok(dyq, xq, N, K, T):
        _wgrad8(g.buf, dyq, xq, N, K, T, s)
        return None
    if g.buf is g.mg and _C.gemm2_supported(1, 1, 7, N, K, T):
        # the common case without any Python stream plumbing: TT GEMM (+ split-K reduce) launched on the side stream
        sp = _C.gemm2_splits(N, K, T)
        # (fp32 atomics per K-split instead of slabs + one reduce pass: headline -5.7 %, bert-large B = 64 -13.5 %,
        # profiles/r6/wgrad_atomic_rejected_r6.log)
        _C.gemm2_on(s.cuda_stream, dy, x, g.buf, 1, 1, 7, None, None, None, 0.0, 0, sp,
                    _workspace(sp * N * K, dy.device, s), None)
        return None
    with torch.cuda.stream(s):
        gemm_wgrad_(g, dy, x, dyq, xq)
        return g.done()


def wgrad_done(g: "_Grad", dy: torch.Tensor, x: torch.Tensor, dyq=None, xq=None):
    """``g += dyᵀ·x`` then ``g.done()`` — on the wgrad side stream when the gradient lands in the flat
    fp32 main_grad buffer (training with a FlatParamStore) and the step is small enough, synchronously otherwise.
    ``dyq`` / ``xq``: the producers' fp8 copies (q, sinv) of dy / x: with both, the fp8 TT kernel runs instead.
    (One fork per weight gradient: deferring the first weight gradient of each block half to the second one's fork,
    one compute-stream event instead of two, measured 0.8 % slower at bert-large B = 8 and 0.2 % at the headline --
    the side stream starts later -- profiles/r6/fork_merge_defer_ab_r6.log.)"""
    s = side_stream(dy.device) if (g.mg is not None and g.buf is g.mg and _use_side_stream(dy.shape[0])) else None
    if s is None:
        gemm_wgrad_(g, dy, x, dyq, xq)
        return g.done()
    parent = _CAPTURE["parent"]
    if parent is not None:
        _CAPTURE["forked"] = True  # a branch of the graph capture, forked from the capture stream itself
    src = parent.cuda_stream if parent is not None else 0
    if not _JOIN_QUEUED[0]:
        # join the compute stream to the side stream when this backward pass finishes
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
        _JOIN_QUEUED[0] = True
        if _SIDE_DELAY_US > 0:
            # ordering test hook (tests/test_gpu_comm.py): stall the side stream before this backward's first weight
            # gradient, so any consumer of main_grad not ordered after the side stream reads it unfinished
            _C.stream_wait(s.cuda_stream, src)
            with torch.cuda.stream(s):
                _C.cu_hog(1, _SIDE_DELAY_US)
    _STASH.append((dy, x, dyq, xq))
    _C.stream_wait(s.cuda_stream, src)
    if parent is None:
        for f in _FORK_LISTENERS:
            f(s)
    return _launch_wgrad(s, g, dy, x, dyq, xq)


def _wgrad_(g: _Grad, dy2d: torch.Tensor, x2d: torch.Tensor) -> None:
    """g += dyᵀ·x  (fp32 accumulate)."""
    g.buf.add_(torch.mm(dy2d.t(), x2d).to(torch.float32))


def _empty(shape, like, dtype=None):
    return torch.empty(shape, dtype=dtype or like.dtype, device=like.device)


# ------------------------------------------------------------------------------------------ optimizer
def adam_step(p, m, v, g, out, decay, step, eps, b1, b2, gscale, lr_wd, coef=None, out_lo=None, zero_grad=False):
    """``coef``: optional fp32 [4] device tensor (step, eps, grad_scale, lr*wd) read by the kernel instead of the
    host scalars (captured HIP-graph steps, train/graph.py). ``out_lo``: with ``out``, the kernel writes the updated
    weights' bf16 hi / lo halves (fp32 compute: the split-product GEMMs' operands, ops/hip32.py). ``zero_grad``: the
    kernel also clears ``g`` after reading it."""
    _C.adam_step(p, m, v, g, out, decay, step, eps, b1, b2, gscale, lr_wd, coef, out_lo, zero_grad)


# ------------------------------------------------------------------------------------------ linear
class _Linear(torch.autograd.Function):
    """y = x Wᵀ + b for the task heads (pooler / classifier / MLM dense): gemm2 when the shape tiles,
    otherwise the library GEMM (e.g. the 2-way classifier)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if x2.dtype == torch.bfloat16 and _nt_ok(x2.shape[0], w.shape[0], x2.shape[1], EPI_BIAS):
            y = gemm_fwd(x2, w, EPI_BIAS, bias=b)
        else:
            y = torch.addmm(b, x2, w.t())
        ctx.save_for_backward(x2, w, b)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, b = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            if dy2.dtype == torch.bfloat16 and _nt_ok(dy2.shape[0], w.shape[1], dy2.shape[1], EPI_STORE):
                dx = gemm_dgrad(dy2, w).view(ctx.xshape)
            else:
                dx = torch.mm(dy2, w).view(ctx.xshape)
        gw, gb = _Grad(w), _Grad(b)
        if dy2.dtype == torch.bfloat16 and _C.gemm2_supported(1, 1, 7, w.shape[0], w.shape[1], dy2.shape[0]):
            gemm_wgrad_(gw, dy2, x2)
        else:
            _wgrad_(gw, dy2, x2)
        if dy2.shape[1] % 8 == 0:
            _C.colsum(dy2, gb.buf)
        else:
            gb.buf.add_(dy2.float().sum(0))
        return dx, gw.done(), gb.done()


def linear(x, w, b):
    return _Linear.apply(x, w, b)


class _LinearGelu(torch.autograd.Function):
    """gelu(x Wᵀ + b): gemm2 with the bias + GELU epilogue (pre-activation and activation out) when the shape tiles;
    backward: GELU' + bias column sums in one kernel, then gemm2 dgrad / wgrad."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if x2.dtype == torch.bfloat16 and _nt_ok(x2.shape[0], w.shape[0], x2.shape[1], EPI_BIAS_GELU):
            g = torch.empty((x2.shape[0], w.shape[0]), dtype=x2.dtype, device=x2.device)
            y = gemm_fwd(x2, w, EPI_BIAS_GELU, bias=b, out2=g)
        else:
            y = torch.addmm(b, x2, w.t())
            g = torch.empty_like(y)
            _C.gelu_fwd(y, g)
        ctx.save_for_backward(x2, w, b, y)
        ctx.xshape = x.shape
        return g.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dg):
        x2, w, b, y = ctx.saved_tensors
        dg2 = dg.reshape(y.shape).contiguous()
        gw, gb = _Grad(w), _Grad(b)
        da = torch.empty_like(y)
        _C.gelu_bwd_colsum(dg2, y, da, gb.buf)
        dx = None
        if ctx.needs_input_grad[0]:
            if da.dtype == torch.bfloat16 and _nt_ok(da.shape[0], w.shape[1], da.shape[1], EPI_STORE):
                dx = gemm_dgrad(da, w).view(ctx.xshape)
            else:
                dx = torch.mm(da, w).view(ctx.xshape)
        if da.dtype == torch.bfloat16 and _C.gemm2_supported(1, 1, 7, w.shape[0], w.shape[1], da.shape[0]):
            gemm_wgrad_(gw, da, x2)
        else:
            _wgrad_(gw, da, x2)
        return dx, gw.done(), gb.done()


def linear_gelu(x, w, b):
    return _LinearGelu.apply(x, w, b)


# ------------------------------------------------------------------------------------------ LN tails
class _DenseResidualLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, res, ln_w, ln_b, eps, p, seed):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        if x2.dtype == torch.bfloat16 and _nt_ok(x2.shape[0], w.shape[0], x2.shape[1], EPI_BIAS):
            y = gemm_fwd(x2, w, EPI_BIAS, bias=b)
        else:
            y = torch.addmm(b, x2, w.t())
        rows, H = y.shape
        z = torch.empty_like(y)
        out = torch.empty_like(y)
        mean = torch.empty(rows, dtype=torch.float32, device=y.device)
        rstd = torch.empty_like(mean)
        _C.ln_fwd(y, res.reshape(rows, H), ln_w, ln_b, z, out, mean, rstd, float(eps), float(p), _s64(seed))
        ctx.save_for_backward(x2, w, b, z, mean, rstd, ln_w, ln_b)
        ctx.p, ctx.seed, ctx.xshape = float(p), seed, x.shape
        return out.view(res.shape)

    @staticmethod
    def backward(ctx, dout):
        x2, w, b, z, mean, rstd, ln_w, ln_b = ctx.saved_tensors
        dout2 = dout.reshape(z.shape).contiguous()
        gw, gb, gg, gbe = _Grad(w), _Grad(b), _Grad(ln_w), _Grad(ln_b)
        dy = torch.empty_like(z)
        if ctx.p > 0:
            dz = torch.empty_like(z)
            _C.ln_bwd(dout2, z, mean, rstd, ln_w, dz, dy, None, gg.buf, gbe.buf, gb.buf, ctx.p, _s64(ctx.seed))
        else:
            _C.ln_bwd(dout2, z, mean, rstd, ln_w, None, dy, None, gg.buf, gbe.buf, gb.buf, 0.0, 0)
            dz = dy
        gln_w, gln_b = gg.done(), gbe.done()
        dx = None
        if ctx.needs_input_grad[0]:
            if _nt_ok(dy.shape[0], w.shape[1], dy.shape[1], EPI_STORE):
                dx = gemm_dgrad(dy, w).view(ctx.xshape)
            else:
                dx = torch.mm(dy, w).view(ctx.xshape)
        if _C.gemm2_supported(1, 1, 7, w.shape[0], w.shape[1], dy.shape[0]):
            gemm_wgrad_(gw, dy, x2)
        else:
            _wgrad_(gw, dy, x2)
        return dx, gw.done(), gb.done(), dz.view(dout.shape), gln_w, gln_b, None, None, None


def dense_residual_ln(x, w, b, residual, ln_w, ln_b, eps, p, seed):
    return _DenseResidualLN.apply(x, w, b, residual, ln_w, ln_b, eps, p, seed)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        rows, H = x2.shape
        out = torch.empty_like(x2)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        _C.ln_fwd(x2, None, w, b, None, out, mean, rstd, float(eps), 0.0, 0)
        ctx.save_for_backward(x2, mean, rstd, w, b)
        return out.view(x.shape)

    @staticmethod
    def backward(ctx, dout):
        x2, mean, rstd, w, b = ctx.saved_tensors
        gg, gbe = _Grad(w), _Grad(b)
        dx = torch.empty_like(x2)
        _C.ln_bwd(dout.reshape(x2.shape).contiguous(), x2, mean, rstd, w, None, dx, None, gg.buf, gbe.buf, None, 0.0, 0)
        return dx.view(dout.shape), gg.done(), gbe.done(), None


def layer_norm(x, w, b, eps):
    return _LayerNorm.apply(x, w, b, eps)


# ------------------------------------------------------------------------------------------ dropout
class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        xc = x.contiguous()
        out = torch.empty_like(xc)
        _C.dropout(xc, out, float(p), _s64(seed))
        ctx.p, ctx.seed = float(p), seed
        return out

    @staticmethod
    def backward(ctx, dout):
        dx = torch.empty_like(dout)
        _C.dropout(dout.contiguous(), dx, ctx.p, _s64(ctx.seed))
        return dx, None, None


def dropout(x, p, seed):
    if x.dtype != torch.bfloat16 or x.dim() == 0 or x.shape[-1] % 4:
        from .reference import dropout as ref

        return ref(x, p, seed, True)
    return _Dropout.apply(x, p, seed)


# ------------------------------------------------------------------------------------------ embeddings
class _EmbedLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, pos_ids, type_ids, word, pos, typ, ln_w, ln_b, eps, p, seed, pos_is_arange, q8_for):
        B, S = ids.shape
        H = word.shape[1]
        ids_c = ids.contiguous().long()
        pos_c = pos_ids.contiguous().long()
        tt_c = type_ids.contiguous().long() if typ is not None else None
        out = torch.empty((B * S, H), dtype=word.dtype, device=word.device)
        mean = torch.empty(B * S, dtype=torch.float32, device=word.device)
        rstd = torch.empty_like(mean)
        # fp8: the first layer's QKV GEMM takes its operand's fp8 copy from this kernel (no separate quantise pass)
        st = _site_ready(q8_for, "_hsd_fp8_x", "_hsd_q")
        if st is not None and H % 8 == 0 and _C.gemm8_supported(EPI_BIAS, B * S, q8_for.shape[0], H):
            q = torch.empty((B * S, H), dtype=torch.uint8, device=word.device)
            sinv = torch.empty(1, dtype=torch.float32, device=word.device)
            _C.embed_fwd(ids_c, pos_c, tt_c, word, pos, typ, ln_w, ln_b, out, mean, rstd, float(eps), float(p),
                         _s64(seed), q, st[0:1], sinv, st[1:2])
            _Q8_HANDOFF.put(out, q, sinv)
        else:
            _C.embed_fwd(ids_c, pos_c, tt_c, word, pos, typ, ln_w, ln_b, out, mean, rstd, float(eps), float(p),
                         _s64(seed))
        ctx.save_for_backward(ids_c, pos_c, tt_c if tt_c is not None else ids_c, word, pos,
                              typ if typ is not None else word, ln_w, ln_b, mean, rstd)
        ctx.has_type = typ is not None
        ctx.p, ctx.seed, ctx.B, ctx.S, ctx.arange = float(p), seed, B, S, bool(pos_is_arange)
        return out.view(B, S, H)

    @staticmethod
    def backward(ctx, dout):
        ids, pos_ids, tt, word, pos, typ, ln_w, ln_b, mean, rstd = ctx.saved_tensors
        gwd, gp, gg, gbe = _Grad(word), _Grad(pos), _Grad(ln_w), _Grad(ln_b)
        gt = _Grad(typ) if ctx.has_type else None
        _C.embed_bwd(dout.contiguous(), ids, pos_ids, tt if ctx.has_type else None, word, pos,
                     typ if ctx.has_type else None, ln_w, mean, rstd, gwd.buf, gp.buf, gt.buf if gt else None,
                     gg.buf, gbe.buf, ctx.B, ctx.S, ctx.arange, ctx.p, _s64(ctx.seed))
        return (None, None, None, gwd.done(), gp.done(), gt.done() if gt else None, gg.done(), gbe.done(),
                None, None, None, None, None)


def embed_ln(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b, eps, p, seed,
             pos_is_arange=False, q8_for=None):
    """``pos_is_arange``: position ids are ``arange(S)`` for every row (BERT/DistilBERT) — enables the
    per-block position-gradient reduction instead of per-token atomics. ``q8_for``: the first encoder layer's QKV
    weight (fp8 path: the kernel also writes the output's fp8 copy for it)."""
    return _EmbedLN.apply(input_ids, position_ids, token_type_ids, word_w, pos_w, type_w, ln_w, ln_b, eps, p, seed,
                          pos_is_arange, q8_for)


# ------------------------------------------------------------------------------------------ attention
def _keep_mask(B, S, heads, p, device):
    """Dropout keep bits the attention forward writes for its backward, which reads them instead of re-hashing every
    (query, key) pair (attention128.hip, attentionS.hip headers): S^2/8 B per (batch, head) (25 MB per bert-base
    layer at B = 1024, S = 128; 4 MB per bert-large layer at B = 8, S = 512). None without dropout or where the
    kernels do not support it."""
    if p > 0:
        n = _C.attn_keep_mask_numel(B, S, heads)
        if n > 0:
            return torch.empty(n, dtype=torch.int32, device=device)
    return None


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, mask_bias, B, S, heads, p, seed):
        qkv = qkv.contiguous()
        H = qkv.shape[-1] // 3
        out = torch.empty((B * S, H), dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B * heads * S, dtype=torch.float32, device=qkv.device)
        mb = mask_bias.contiguous().float() if mask_bias is not None else None
        km = _keep_mask(B, S, heads, p, qkv.device)
        _C.attn_fwd(qkv, mb, out, lse, B, S, heads, float(p), _s64(seed), km)
        ctx.save_for_backward(qkv, out, lse, mb if mb is not None else lse, km if km is not None else lse)
        ctx.has_mask, ctx.has_km = mb is not None, km is not None
        ctx.B, ctx.S, ctx.heads, ctx.p, ctx.seed = B, S, heads, float(p), seed
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, mb, km = ctx.saved_tensors
        dqkv = torch.empty_like(qkv)
        dq_acc = _attn_ws(ctx.B, ctx.S, ctx.heads, out.device)
        _C.attn_bwd(qkv, mb if ctx.has_mask else None, out, dout.contiguous(), lse, dqkv, dq_acc, ctx.B, ctx.S,
                    ctx.heads, ctx.p, _s64(ctx.seed), None, km if ctx.has_km else None)
        return dqkv, None, None, None, None, None, None


def _attn_ws(B, S, heads, device):
    """fp32 scratch of the attention backward for S > 128 (delta rows of the streaming kernels, or the
    zeroed dQ accumulator of the generic one)."""
    n, zero = _C.attn_bwd_ws(B, S, heads)
    if n == 0:
        return None
    return (torch.zeros if zero else torch.empty)(n, dtype=torch.float32, device=device)


def attention(qkv, mask_bias, batch, seq, heads, p, seed):
    if qkv.shape[-1] != 3 * heads * 64:
        from .reference import attention as ref

        return ref(qkv, mask_bias, batch, seq, heads, p, seed, p > 0)
    return _Attention.apply(qkv, mask_bias, batch, seq, heads, p, seed)


# ------------------------------------------------------------------------------------------ GEMM helpers
EPI_STORE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_DROP_RES, EPI_RES, EPI_DGELU, EPI_F32_ATOMIC = range(7)
EPI_F32_SLAB, EPI_BIAS_GELU_D, EPI_MUL, EPI_STORE_RDOT = 7, 8, 9, 10  # gemm2 only

# split-K factors for the wgrad GEMM (fp32 atomic epilogue), measured with tools/bench_gemm.py at
# T = 32768 tokens; key = (out_features, in_features)
_WGRAD_SPLITS = {(2304, 768): 4, (768, 768): 8, (3072, 768): 8, (768, 3072): 8,
                 (3072, 1024): 8, (1024, 4096): 8, (1024, 1024): 8, (4096, 1024): 8}


def _wgrad_splits(n_out: int, k_in: int, tokens: int) -> int:
    s = _WGRAD_SPLITS.get((n_out, k_in))
    if s is None:
        tiles = -(-n_out // 256) * -(-k_in // 128)
        s = 1
        while tiles * s * 2 <= 512 and s < 16:
            s *= 2
    # keep >= 2 k-tiles (64 tokens each) per split
    while s > 1 and tokens // s < 128:
        s //= 2
    return s


_WS = {}


def _workspace(numel: int, device, stream=None) -> torch.Tensor:
    """Split-K slab workspace (fp32), grown on demand, reused stream-ordered across wgrad GEMMs. One buffer PER STREAM
    (``stream``: the stream that will use it; default the current one): the side-stream weight gradients and the
    compute-stream ones never share slabs, and a grown buffer is allocated from its own stream's pool, so the old one
    goes back to the pool of the only stream that used it (no cross-stream reuse while a kernel still writes it)."""
    sid = stream.cuda_stream if stream is not None else torch.cuda.current_stream(device).cuda_stream
    key = (device.type, device.index, sid)
    buf = _WS.get(key)
    if buf is None or buf.numel() < numel:
        if stream is not None:
            with torch.cuda.stream(stream):
                buf = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        else:
            buf = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        _WS[key] = buf
    return buf


def _nt_ok(M, N, K, epi):
    return _C.gemm2_supported(0, 0, epi, M, N, K)


# ---- fp8 GEMM path (gemm8.hip / fp8.hip) -------------------------------------------
# With fp8 on, the forward and dgrad GEMMs of every weight the FlatParamStore keeps an fp8 copy of (the
# encoder's qkv / attn_out / ffn1 / ffn2) run on the fp8 MFMA kernel: the activation (forward) or the
# incoming gradient (dgrad) is quantised per tensor on the device, the weight copies are re-quantised
# once per optimizer step. Weight gradients stay bf16 x bf16 -> fp32 (gemm2 TT), as do the task heads.
FP8_E4M3, FP8_E5M2 = 0, 1
_FP8 = {"on": False, "grad_fmt": FP8_E4M3}


def set_fp8(on: bool, grad_fmt: str = "e4m3") -> None:
    _FP8["on"] = bool(on)
    _FP8["grad_fmt"] = FP8_E5M2 if grad_fmt == "e5m2" else FP8_E4M3


def fp8_enabled() -> bool:
    return _FP8["on"]


def quant_fp8(x: torch.Tensor, fmt: int = FP8_E4M3, state: Optional[torch.Tensor] = None):
    """(q uint8 [same shape], sinv fp32 [1]) with q = sat(x · FMT_MAX / amax), sinv = amax / FMT_MAX.

    ``state`` None: current scaling (amax of x, two passes). Otherwise a delayed-scaling site, fp32 [2] =
    (amax scaling this step, running amax of this step — rolled by FlatParamStore.refresh_fp8): one pass;
    the site's first use calibrates with the amax pass."""
    x = x.contiguous()
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    if state is None:
        sc = torch.zeros(2, dtype=torch.float32, device=x.device)  # [amax, sinv]
        _C.fp8_quant(x, sc[0:1], q, sc[1:2], fmt, True)
        return q, sc[1:2]
    sinv = torch.empty(1, dtype=torch.float32, device=x.device)
    calibrated = getattr(state, "_hsd_cal", False)
    _C.fp8_quant(x, state[0:1], q, sinv, fmt, not calibrated, state[1:2])
    state._hsd_cal = True
    return q, sinv


def _fp8_w(w, attr):
    if not _FP8["on"]:
        return None
    return getattr(w, attr, None)


# fp8 copies written by the producing LayerNorm (fused quantisation, no standalone quant pass): the LN at the end of
# a block quantises its output for the NEXT block's first GEMM with that GEMM's delayed-scaling site, and the LN
# backward quantises dy for the block's own fp8 dgrad. A site is fused only once it is calibrated (its first use
# runs the standalone amax + quant passes), so fused and standalone paths give the same bytes.
class _Q8Handoff:
    """One producer-written fp8 copy waiting for the GEMM that consumes the producer's output.

    The producer (LayerNorm fwd / bwd, a GEMM epilogue) calls :meth:`put` with its bf16 output; the next GEMM calls
    :meth:`take` with its input. The copy is handed over only if that input IS the producer's output (same memory,
    same size) and the output is still alive and unmodified: a weak reference to the producer's tensor (a view keeps
    its base alive, so a dead reference means the memory may have been reused by another tensor) and the tensor's
    version counter (bumped by any in-place write). One slot: only the immediately following GEMM may take it."""

    def __init__(self):
        self._slot = None

    def put(self, out: torch.Tensor, q: torch.Tensor, sinv: torch.Tensor) -> None:
        self._slot = (weakref.ref(out), out.data_ptr(), out.numel(), out._version, q, sinv)

    def take(self, x: torch.Tensor):
        s, self._slot = self._slot, None
        if s is None:
            return None
        ref, ptr, numel, ver, q, sinv = s
        out = ref()
        if out is None or out._version != ver or x.data_ptr() != ptr or x.numel() != numel:
            return None
        return q, sinv

    def clear(self) -> None:
        self._slot = None


_Q8_HANDOFF = _Q8Handoff()


def _site_ready(w, state_attr: str, wattr: str):
    """The calibrated delayed-scaling state of ``w``'s fp8 site, or None (fp8 off / no fp8 copy / first use)."""
    if w is None or not _FP8["on"] or getattr(w, wattr, None) is None:
        return None
    st = getattr(w, state_attr, None)
    return st if st is not None and getattr(st, "_hsd_cal", False) else None


def _dequant8(q8, fmt: int, like: torch.Tensor) -> torch.Tensor:
    """bf16 values of an fp8 copy (q, sinv): the fallback for a consumer that needs the bf16 twin a ``q8_only``
    epilogue did not store (a path change between forward and backward, a retained-graph second backward)."""
    q, sinv = q8
    f8 = torch.float8_e5m2 if fmt == FP8_E5M2 else torch.float8_e4m3fn
    return (q.view(f8).to(torch.float32) * sinv).to(like.dtype).view(like.shape)


def _fp8_fwd_ok(w, epi, M: int, K: int) -> bool:
    """The forward GEMM of ``w`` on an [M, K] input runs on the fp8 kernel (gemm_fwd's first branch)."""
    return _fp8_w(w, "_hsd_q") is not None and _C.gemm8_supported(epi, M, w.shape[0], K)


def _fp8_dgrad_ok(w, epi, M: int) -> bool:
    """The dgrad of ``w`` for an [M, N_out] incoming gradient runs on the fp8 kernel (gemm_dgrad's first branch)."""
    return _fp8_w(w, "_hsd_qt") is not None and _C.gemm8_supported(epi, M, w.shape[1], w.shape[0])


def _take_q8(x):
    """The fp8 copy a producer wrote for activation ``x`` (:class:`_Q8Handoff`), or None."""
    return _Q8_HANDOFF.take(x)


def _q8_out(like, w, state_attr: str, wattr: str, fmt: int):
    """Buffers for a producer-written fp8 copy of ``like`` for ``w``'s calibrated site, or None."""
    st = _site_ready(w, state_attr, wattr)
    if st is None:
        return None
    q = torch.empty(like.shape, dtype=torch.uint8, device=like.device)
    return q, torch.empty(1, dtype=torch.float32, device=like.device), st, fmt


def _q8_kw(q8):
    if q8 is None:
        return {}
    q, sinv, st, fmt = q8
    return {"q8": q, "q8_amax": st[0:1], "q8_sinv": sinv, "q8_track": st[1:2], "q8fmt": fmt}


def gemm_fwd(x, w, epi, bias=None, aux=None, out2=None, p=0.0, seed=0, xq=None, q8_for=None, q8_only=False):
    """y[T, N] = x[T, K] · w[N, K]ᵀ with epilogue (gemm2 8-phase kernel; 128-tile kernel for odd shapes;
    gemm8 fp8 kernel when fp8 is on and the weight has an fp8 copy). ``xq``: x's fp8 copy (q, sinv) already
    written by its producer. ``q8_for``: the weight of the fp8 GEMM that consumes the output (``out2`` for the
    two-output GELU epilogue): on the fp8 path the epilogue writes that GEMM's fp8 input copy too. ``q8_only``: the
    caller's consumers of ``out2`` all take that fp8 copy, so its bf16 values are not stored when the copy is written
    (returned ``y`` then carries ``_hsd_q8_only = True``; ``out2``'s contents are undefined)."""
    y = torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
    wq = _fp8_w(w, "_hsd_q")
    if wq is not None and _C.gemm8_supported(epi, x.shape[0], w.shape[0], x.shape[1]):
        qx, sx = xq if xq is not None else quant_fp8(x, FP8_E4M3, getattr(w, "_hsd_fp8_x", None))
        q8 = _q8_out(y, q8_for, "_hsd_fp8_x", "_hsd_q", FP8_E4M3) \
            if q8_for is not None and epi in (EPI_BIAS_GELU, EPI_BIAS_GELU_D) and out2 is not None else None
        only = bool(q8_only and q8 is not None)
        _C.gemm8(qx, FP8_E4M3, sx, wq, FP8_E4M3, w._hsd_qs, y, epi, bias, aux, out2, float(p), _s64(seed), None,
                 **_q8_kw(q8), q8_only=only)
        if q8 is not None:
            _Q8_HANDOFF.put(out2, q8[0], q8[1])
        if only:
            y._hsd_q8_only = True
        return y
    if _nt_ok(x.shape[0], w.shape[0], x.shape[1], epi):
        _C.gemm2(x, w, y, 0, 0, epi, bias, aux, out2, float(p), _s64(seed), 0, None, None)  # 0: auto split-K
    else:
        _C.gemm(x, w, y, 0, 0, epi, bias, aux, out2, float(p), _s64(seed), 1)
    return y


def gemm_dgrad_rd(dy, w, o, rd, seq, dyq=None):
    """The out-projection dgrad dx = dy · w (the attention backward's dO) whose epilogue also writes the streaming
    attention backward's delta rows rd[(b·heads + h)·S + s] = Σ_head dx·o (E2_STORE_RDOT; gemm_common.h), so the
    backward skips its own delta pass (re-reading dO and O, one more launch). fp8 weights: the fp8 persistent kernel
    (dy's fp8 copy ``dyq``, or quantised here like gemm_dgrad). Returns ``(dx, True)``, or
    ``(gemm_dgrad(dy, w, dyq=dyq), False)`` when no kernel path takes the shape (N % 256)."""
    M, N, K = dy.shape[0], w.shape[1], dy.shape[1]
    wqt = _fp8_w(w, "_hsd_qt")
    if wqt is not None and o.is_contiguous() and o.shape == (M, N) and \
            _C.gemm8_supported(EPI_STORE_RDOT, M, N, K):
        fmt = _FP8["grad_fmt"]
        qdy, sdy = dyq if dyq is not None else quant_fp8(dy, fmt, getattr(w, "_hsd_fp8_g", None))
        dx = torch.empty((M, N), dtype=dy.dtype, device=dy.device)
        _C.gemm8(qdy, fmt, sdy, wqt, FP8_E4M3, w._hsd_qs, dx, EPI_STORE_RDOT, None, o, None, 0.0, 0, None, rd=rd,
                 rd_seq=seq)
        return dx, True
    if wqt is None and o.is_contiguous() and o.shape == (M, N):
        wt = getattr(w, "_hsd_wt", None)
        if wt is not None and (wt.shape[0] != N or wt.shape[1] != K):
            wt = None
        if wt is None and w.is_contiguous() and _C.gemm2_supported(0, 1, EPI_STORE_RDOT, M, N, K):
            dx = torch.empty((M, N), dtype=dy.dtype, device=dy.device)
            _C.gemm2(dy, w, dx, 0, 1, EPI_STORE_RDOT, None, o, None, 0.0, 0, 0, None, None, rd, seq)
            return dx, True
        if wt is not None and _C.gemm2_supported(0, 0, EPI_STORE_RDOT, M, N, K):
            dx = torch.empty((M, N), dtype=dy.dtype, device=dy.device)
            _C.gemm2(dy, wt, dx, 0, 0, EPI_STORE_RDOT, None, o, None, 0.0, 0, 0, None, None, rd, seq)
            return dx, True
    return gemm_dgrad(dy, w, dyq=dyq), False


def gemm_dgrad(dy, w, epi=EPI_STORE, aux=None, dbias=None, dyq=None, q8_for=None, q8_only=False):
    """dx[T, K] = dy[T, N] · w[N, K]  (NT kernel on the transposed weight wᵀ [K, N]).

    ``dbias`` (DGELU only): fp32 [K] buffer that receives the column sums of dx (the bias gradient of
    the layer that produced ``aux``) from the epilogue; returns ``(dx, fused)``-style via attribute.
    ``q8_only``: every consumer of dx takes the fp8 copy written for ``q8_for``, so dx's bf16 values are not stored
    when that copy is written (dx then carries ``_hsd_q8_only = True`` and its contents are undefined)."""
    dx = torch.empty((dy.shape[0], w.shape[1]), dtype=dy.dtype, device=dy.device)
    wqt = _fp8_w(w, "_hsd_qt")
    if wqt is not None and _C.gemm8_supported(epi, dy.shape[0], w.shape[1], dy.shape[1]):
        fuse = dbias is not None and epi in (EPI_DGELU, EPI_MUL) and w.shape[1] % 256 == 0
        fmt = _FP8["grad_fmt"]
        qdy, sdy = dyq if dyq is not None else quant_fp8(dy, fmt, getattr(w, "_hsd_fp8_g", None))
        # q8_for: the next fp8 dgrad's weight -- the epilogue writes its dy copy (the GELU'-product output)
        q8 = _q8_out(dx, q8_for, "_hsd_fp8_g", "_hsd_qt", fmt) \
            if q8_for is not None and epi in (EPI_MUL, EPI_DGELU) else None
        # the bias-gradient column sums read dx when they are not fused: then dx's bf16 values must exist
        only = bool(q8_only and q8 is not None and (dbias is None or fuse))
        _C.gemm8(qdy, fmt, sdy, wqt, FP8_E4M3, w._hsd_qs, dx, epi, None, aux, None, 0.0, 0, dbias if fuse else None,
                 **_q8_kw(q8), q8_only=only)
        if only:
            dx._hsd_q8_only = True
        if dbias is not None and not fuse:
            _C.colsum(dx, dbias)
        if q8 is not None:
            _Q8_HANDOFF.put(dx, q8[0], q8[1])
        return dx
    wt = getattr(w, "_hsd_wt", None)  # FlatParamStore keeps Wᵀ fresh (one batched transpose per step)
    if wt is not None and (wt.shape[0] != w.shape[1] or wt.shape[1] != w.shape[0]):
        wt = None
    fuse = dbias is not None and epi in (EPI_DGELU, EPI_MUL) and w.shape[1] % 256 == 0
    if wt is None and w.is_contiguous() and _C.gemm2_supported(0, 1, epi, dy.shape[0], w.shape[1], dy.shape[1]):
        # no stored Wᵀ (small steps): the NT kernel reads W [N_out][K_in] itself as its k-strided B operand
        _C.gemm2(dy, w, dx, 0, 1, epi, None, aux, None, 0.0, 0, 0, None, dbias if fuse else None)
        if dbias is not None and not fuse:
            _C.colsum(dx, dbias)
    elif _nt_ok(dy.shape[0], w.shape[1], dy.shape[1], epi):
        if wt is None:
            wt = w.t().contiguous()
        _C.gemm2(dy, wt, dx, 0, 0, epi, None, aux, None, 0.0, 0, 0, None, dbias if fuse else None)
        if dbias is not None and not fuse:
            _C.colsum(dx, dbias)
    else:
        _C.gemm(dy, w, dx, 0, 1, epi, None, aux, None, 0.0, 0, 1)
        if dbias is not None:
            _C.colsum(dx, dbias)
    return dx


# fp8 weight gradients (BASELINE.json configs[4]): when both operands of a weight gradient already have an fp8 copy
# written by their producers (the fp8 forward / dgrad path's delayed-scaling sites), dW += dyᵀ·x runs on the fp8 TT
# kernel (gemm2.hip gemm8tt_kernel: both copies read as written, transposed in LDS) instead of the bf16 one.
# HSD_FP8_WGRAD=0 keeps the weight gradients bf16 under --fp8.
_FP8_WGRAD = _os.environ.get("HSD_FP8_WGRAD", "1") == "1"
WGRAD8_CALLS = [0]  # fp8 weight-gradient launches (tests)
# fp8 FFN: epilogues whose bf16 output is only ever read through its fp8 copy skip the bf16 store (tests switch it off
# to compare against the path that writes both)
_Q8_ONLY = True


def _wgrad8_ok(dyq, xq, N, K, T) -> bool:
    return (_FP8["on"] and _FP8_WGRAD and dyq is not None and xq is not None
            and _C.gemm8_wgrad_supported(N, K, T))


# Side-stream fp8 weight gradients take 2 token splits instead of the kernel's cost model, which plans for a GPU of its
# own (4-16 splits at roberta-large T = 32,768: every CU busy, one fp32 M x N slab written and re-read per split). The
# side stream shares the GPU with the dgrad chain: roberta-large MLM fp8 +3.1 % (1,101-1,107 vs 1,068-1,072 seq/s; 3
# splits, and the model's count halved, in between; 1 split -11 %). The bf16 TT kernel is the opposite: the headline is
# 7 % slower at half its model's splits (profiles/r6/fp8_wgrad_splits_ab_r6.log, wgrad_splits_side_stream_ab_r6.log).
# (Splits for ~64 / 128 / 192 workgroups per GEMM instead of a fixed 2: -3 % / within noise / -1 %,
# profiles/r6/fp8_wgrad_side_wgs_ab_r6.log.)
_WGRAD8_SIDE_SPLITS = 2


def _wgrad8(buf, dyq, xq, N, K, T, stream=None) -> None:
    """buf[N, K] += dequant(dyq)ᵀ · dequant(xq) on ``stream`` (None: the current stream)."""
    sp = _WGRAD8_SIDE_SPLITS if stream is not None and T >= 2 * 128 * _WGRAD8_SIDE_SPLITS else 0
    ws = _workspace(_C.gemm8_wgrad_ws_numel(N, K, T, sp), buf.device, stream)
    _C.gemm8_wgrad(stream.cuda_stream if stream is not None else 0, dyq[0], _FP8["grad_fmt"], dyq[1], xq[0],
                   FP8_E4M3, xq[1], buf, sp, ws)
    WGRAD8_CALLS[0] += 1


def gemm_wgrad_(g: "_Grad", dy, x, dyq=None, xq=None):
    """g.buf[N, K] += dy[T, N]ᵀ · x[T, K]   (fp32; split-K over tokens into slabs + one reduce). With the fp8 copies
    ``dyq`` / ``xq`` (q, sinv) of both operands: the fp8 TT kernel on them."""
    N, K, T = dy.shape[1], x.shape[1], dy.shape[0]
    if _wgrad8_ok(dyq, xq, N, K, T):
        _wgrad8(g.buf, dyq, xq, N, K, T)
    elif _C.gemm2_supported(1, 1, 7, N, K, T):
        sp = _C.gemm2_splits(N, K, T)
        ws = _workspace(sp * N * K, dy.device)
        _C.gemm2(dy, x, g.buf, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)
    else:
        splits = _wgrad_splits(N, K, T)
        _C.gemm(dy, x, g.buf, 1, 1, EPI_F32_ATOMIC, None, None, None, 0.0, 0, splits)


def _ln_fwd(z, w, b, eps, q8_for=None):
    """LayerNorm forward; with ``q8_for`` (the next GEMM's weight) on a calibrated fp8 site, the kernel also writes
    the output's fp8 copy, which the next block's first GEMM picks up (:func:`_take_q8`)."""
    rows, H = z.shape
    out = torch.empty_like(z)
    mean = torch.empty(rows, dtype=torch.float32, device=z.device)
    rstd = torch.empty_like(mean)
    st = _site_ready(q8_for, "_hsd_fp8_x", "_hsd_q")
    if st is not None and H % 8 == 0 and H <= 1024 and _C.gemm8_supported(EPI_BIAS, rows, q8_for.shape[0], H):
        q = torch.empty((rows, H), dtype=torch.uint8, device=z.device)
        sinv = torch.empty(1, dtype=torch.float32, device=z.device)
        _C.ln_fwd_q8(z, w, b, out, mean, rstd, float(eps), q, st[0:1], sinv, st[1:2])
        _Q8_HANDOFF.put(out, q, sinv)
    else:
        _C.ln_fwd(z, None, w, b, None, out, mean, rstd, float(eps), 0.0, 0)
    return out, mean, rstd


def _ln_bwd(dout2, z, mean, rstd, ln_w, dz, dy, g_lnw, g_lnb, g_b, p, seed, consumer_w, q8_only=False):
    """LN backward into dy (and dz with dropout); returns dy's fp8 copy (q, sinv) when ``consumer_w``'s dgrad runs
    fp8 on a calibrated site (quantised in the same pass), else None. ``q8_only`` (dropout on, so dz is its own
    buffer): every consumer of dy takes that fp8 copy, and dy's bf16 values are not stored."""
    st = _site_ready(consumer_w, "_hsd_fp8_g", "_hsd_qt")
    rows, H = z.shape
    if st is not None and H <= 1024 and _C.gemm8_supported(EPI_STORE, rows, consumer_w.shape[1], H):
        q = torch.empty((rows, H), dtype=torch.uint8, device=z.device)
        sinv = torch.empty(1, dtype=torch.float32, device=z.device)
        _C.ln_bwd_q8(dout2, z, mean, rstd, ln_w, dz, dy, g_lnw.buf, g_lnb.buf, g_b.buf, p, _s64(seed) if p > 0 else 0,
                     q, st[0:1], sinv, st[1:2], _FP8["grad_fmt"], q8_only=bool(q8_only and p > 0 and dz is not None))
        return q, sinv
    _C.ln_bwd(dout2, z, mean, rstd, ln_w, dz, dy, None, g_lnw.buf, g_lnb.buf, g_b.buf, p, _s64(seed) if p > 0 else 0)
    return None


# ------------------------------------------------------------------------------------------ fused blocks
class _AttnBlock(torch.autograd.Function):
    """h1 = LN(dropout(attn(h Wqkvᵀ + b) Woᵀ + bo) + h) with a hand-written backward:
    LN-bwd (+dropout, + out-proj bias grad) -> Wo wgrad / dgrad -> flash-attn bwd -> bias colsum ->
    Wqkv wgrad -> dgrad with the residual gradient added in the GEMM epilogue."""

    @staticmethod
    def forward(ctx, h, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, eps, mask_bias, B, S, heads, p_a, seed_a, p_h,
                seed_h, q8_next=None):
        h2d = h.reshape(-1, h.shape[-1])
        hq = _take_q8(h2d)
        qkv = gemm_fwd(h2d, qkv_w, EPI_BIAS, bias=qkv_b, xq=hq)
        H = out_w.shape[0]
        actx = torch.empty((h2d.shape[0], H), dtype=h.dtype, device=h.device)
        lse = torch.empty(B * heads * S, dtype=torch.float32, device=h.device)
        mb = mask_bias.contiguous().float() if mask_bias is not None else None
        xq = None
        st = _site_ready(out_w, "_hsd_fp8_x", "_hsd_q")
        if st is not None and _C.attn_q8_supported(S) and _C.gemm8_supported(EPI_BIAS_DROP_RES, h2d.shape[0], H, H):
            # the attention kernel writes the context's fp8 copy for the fp8 out-projection (no quant pass)
            q = torch.empty((h2d.shape[0], H), dtype=torch.uint8, device=h.device)
            sinv = torch.empty(1, dtype=torch.float32, device=h.device)
            km = _keep_mask(B, S, heads, p_a, h.device)
            _C.attn_fwd_q8(qkv, mb, actx, lse, B, S, heads, float(p_a), _s64(seed_a), q, st[0:1], sinv, st[1:2], km)
            xq = (q, sinv)
        else:
            km = _keep_mask(B, S, heads, p_a, h.device)
            _C.attn_fwd(qkv, mb, actx, lse, B, S, heads, float(p_a), _s64(seed_a), km)
        z = gemm_fwd(actx, out_w, EPI_BIAS_DROP_RES, bias=out_b, aux=h2d, p=p_h, seed=seed_h, xq=xq)
        out, mean, rstd = _ln_fwd(z, ln_w, ln_b, eps, q8_for=q8_next)
        ctx.save_for_backward(h2d, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, qkv, actx, lse, z, mean, rstd,
                              mb if mb is not None else lse, km if km is not None else lse)
        ctx.cfg = (B, S, heads, float(p_a), seed_a, float(p_h), seed_h, mb is not None)
        ctx.has_km = km is not None
        # fp8 copies of the weight gradients' activation operands (kept only on the fp8 weight-gradient path)
        ctx.q8 = (hq, xq) if _FP8_WGRAD else (None, None)
        return out.view(h.shape)

    @staticmethod
    def backward(ctx, dout):
        (h2d, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, qkv, actx, lse, z, mean, rstd, mb, km) = ctx.saved_tensors
        B, S, heads, p_a, seed_a, p_h, seed_h, has_mask = ctx.cfg
        dout2 = dout.reshape(z.shape).contiguous()
        g_lnw, g_lnb, g_ow, g_ob = _Grad(ln_w), _Grad(ln_b), _Grad(out_w), _Grad(out_b)
        dy = torch.empty_like(z)
        dz = torch.empty_like(z) if p_h > 0 else None
        # the fp8 copies are released after the first backward (a retained-graph second backward runs bf16)
        hq, actq = ctx.q8 or (None, None)
        ctx.q8 = None
        T, H = z.shape
        # dy's consumers (the out-projection weight gradient with the context's fp8 copy, its dgrad) both fp8: the LN
        # backward stores only dy's fp8 copy
        dy_q8 = bool(_Q8_ONLY and _FP8["on"] and _FP8_WGRAD and actq is not None and _C.gemm8_wgrad_supported(H, H, T)
                     and _fp8_dgrad_ok(out_w, EPI_STORE, T))
        dyq = _ln_bwd(dout2, z, mean, rstd, ln_w, dz, dy, g_lnw, g_lnb, g_ob, p_h, seed_h, out_w, q8_only=dy_q8)
        if dz is None:
            dz = dy
        r_lnw, r_lnb, r_ob = g_lnw.done(), g_lnb.done(), g_ob.done()
        r_ow = wgrad_done(g_ow, dy, actx, dyq, actq)
        dq_acc = _attn_ws(B, S, heads, actx.device)
        delta_ready = False
        if dq_acc is not None and dq_acc.numel() == B * heads * S:
            # streaming attention backward: its delta rows come out of this dgrad's epilogue
            dctx, delta_ready = gemm_dgrad_rd(dy, out_w, actx, dq_acc, S, dyq=dyq)
        else:
            dctx = gemm_dgrad(dy, out_w, dyq=dyq)
        dqkv = torch.empty_like(qkv)
        g_qw, g_qb = _Grad(qkv_w), _Grad(qkv_b)
        # the QKV bias gradient (column sums of dqkv) comes out of the attention backward itself
        st = _site_ready(qkv_w, "_hsd_fp8_g", "_hsd_qt") if ctx.needs_input_grad[0] else None
        dqq = None
        if st is not None and _C.attn_q8_supported(S) and _C.gemm8_supported(EPI_RES, dqkv.shape[0], qkv_w.shape[1],
                                                                              dqkv.shape[1]):
            # ... and so does dqkv's fp8 copy for the fp8 QKV dgrad
            q = torch.empty(dqkv.shape, dtype=torch.uint8, device=dqkv.device)
            sinv = torch.empty(1, dtype=torch.float32, device=dqkv.device)
            # dqkv's consumers (the QKV weight gradient with h's fp8 copy, the QKV dgrad) both fp8: only its fp8 copy
            dq_only = bool(_Q8_ONLY and _FP8_WGRAD and hq is not None
                           and _C.gemm8_wgrad_supported(qkv_w.shape[0], qkv_w.shape[1], dqkv.shape[0])
                           and _fp8_dgrad_ok(qkv_w, EPI_RES, dqkv.shape[0]))
            _C.attn_bwd_q8(qkv, mb if has_mask else None, actx, dctx, lse, dqkv, dq_acc, B, S, heads, p_a,
                           _s64(seed_a), g_qb.buf, q, st[0:1], sinv, st[1:2], _FP8["grad_fmt"],
                           km if ctx.has_km else None, delta_ready, q8_only=dq_only)
            dqq = (q, sinv)
        else:
            _C.attn_bwd(qkv, mb if has_mask else None, actx, dctx, lse, dqkv, dq_acc, B, S, heads, p_a, _s64(seed_a),
                        g_qb.buf, km if ctx.has_km else None, delta_ready)
        r_qb = g_qb.done()
        r_qw = wgrad_done(g_qw, dqkv, h2d, dqq, hq)
        dh = gemm_dgrad(dqkv, qkv_w, EPI_RES, aux=dz, dyq=dqq) if ctx.needs_input_grad[0] else None
        return (dh.view(dout.shape) if dh is not None else None, r_qw, r_qb, r_ow, r_ob, r_lnw, r_lnb,
                None, None, None, None, None, None, None, None, None, None)


def attn_block(h, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, eps, mask_bias, B, S, heads, p_a, seed_a, p_h, seed_h,
               q8_next=None):
    """``q8_next``: the weight of the GEMM that consumes this block's output (the FFN's W1): its fp8 input copy is
    written by this block's LayerNorm."""
    return _AttnBlock.apply(h, qkv_w, qkv_b, out_w, out_b, ln_w, ln_b, eps, mask_bias, B, S, heads, p_a, seed_a,
                            p_h, seed_h, q8_next)


class _FFNBlock(torch.autograd.Function):
    """h2 = LN(dropout(gelu(h W1ᵀ + b1) W2ᵀ + b2) + h). Forward: 2 GEMMs (bias+GELU epilogue writing
    pre-activation and activation; bias+dropout+residual epilogue) + LN. Backward: LN-bwd (+dropout,
    + b2 grad) -> W2 wgrad -> dgrad with gelu' epilogue -> b1 colsum -> W1 wgrad -> dgrad + residual."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, ln_w, ln_b, eps, p, seed, q8_next=None):
        h2d = h.reshape(-1, h.shape[-1])
        xq = _take_q8(h2d)
        act = torch.empty((h2d.shape[0], w1.shape[0]), dtype=h.dtype, device=h.device)
        # keep gelu'(pre) instead of pre when the gemm2 path handles both FFN GEMMs: the FFN2 dgrad
        # epilogue is then a product (no erf/exp per element in backward)
        keep_grad = _nt_ok(h2d.shape[0], w1.shape[0], h2d.shape[1], EPI_BIAS_GELU_D) and \
            _nt_ok(h2d.shape[0], w1.shape[0], w2.shape[0], EPI_MUL)
        T, H, I = h2d.shape[0], h2d.shape[1], w1.shape[0]
        # fp8: the activation's bf16 values are not stored when both of its consumers take its fp8 copy -- the FFN2
        # forward (fp8 kernel) and the W2 weight gradient (fp8 TT kernel, with the LN backward's fp8 copy of dy on a
        # calibrated site): 2·T·I bytes of epilogue stores less per layer
        act_q8 = bool(_Q8_ONLY and _FP8["on"] and _FP8_WGRAD and _fp8_fwd_ok(w2, EPI_BIAS_DROP_RES, T, I)
                      and _site_ready(w2, "_hsd_fp8_g", "_hsd_qt") is not None and H <= 1024
                      and _C.gemm8_supported(EPI_STORE, T, I, H) and _C.gemm8_wgrad_supported(H, I, T))
        pre = gemm_fwd(h2d, w1, EPI_BIAS_GELU_D if keep_grad else EPI_BIAS_GELU, bias=b1, out2=act, xq=xq, q8_for=w2,
                       q8_only=act_q8)
        actq = _take_q8(act)
        act_missing = getattr(pre, "_hsd_q8_only", False)
        if act_missing and actq is None:
            raise RuntimeError("FFN forward: the activation's fp8 copy was not handed over")
        z = gemm_fwd(act, w2, EPI_BIAS_DROP_RES, bias=b2, aux=h2d, p=p, seed=seed, xq=actq)
        out, mean, rstd = _ln_fwd(z, ln_w, ln_b, eps, q8_for=q8_next)
        ctx.save_for_backward(h2d, w1, b1, w2, b2, ln_w, ln_b, pre, act, z, mean, rstd)
        ctx.cfg = (float(p), seed, keep_grad)
        ctx.act_missing = act_missing
        ctx.q8 = (xq, actq) if _FP8_WGRAD else (None, None)
        return out.view(h.shape)

    @staticmethod
    def backward(ctx, dout):
        h2d, w1, b1, w2, b2, ln_w, ln_b, pre, act, z, mean, rstd = ctx.saved_tensors
        p, seed, keep_grad = ctx.cfg
        dout2 = dout.reshape(z.shape).contiguous()
        g_lnw, g_lnb, g_w2, g_b2 = _Grad(ln_w), _Grad(ln_b), _Grad(w2), _Grad(b2)
        dy = torch.empty_like(z)
        dz = torch.empty_like(z) if p > 0 else None
        # the fp8 copies are released after the first backward (a retained-graph second backward runs bf16), unless
        # the forward did not store the activation's bf16 values: then its fp8 copy stays for any later backward
        hq, actq = ctx.q8 or (None, None)
        if not ctx.act_missing:
            ctx.q8 = None
        T, H, I = h2d.shape[0], h2d.shape[1], w1.shape[0]
        # dy's consumers (the W2 weight gradient with the activation's fp8 copy, the W2 dgrad) both fp8: the LN
        # backward stores only dy's fp8 copy
        dy_q8 = bool(_Q8_ONLY and _FP8["on"] and _FP8_WGRAD and actq is not None and _C.gemm8_wgrad_supported(H, I, T)
                     and _fp8_dgrad_ok(w2, EPI_MUL if keep_grad else EPI_DGELU, T))
        dyq = _ln_bwd(dout2, z, mean, rstd, ln_w, dz, dy, g_lnw, g_lnb, g_b2, p, seed, w2, q8_only=dy_q8)
        if dz is None:
            dz = dy
        r_lnw, r_lnb, r_b2 = g_lnw.done(), g_lnb.done(), g_b2.done()
        if ctx.act_missing and not _wgrad8_ok(dyq, actq, H, I, T):
            act = _dequant8(actq, FP8_E4M3, act)  # the W2 weight gradient runs bf16 after all
        r_w2 = wgrad_done(g_w2, dy, act, dyq, actq)
        g_w1, g_b1 = _Grad(w1), _Grad(b1)
        # fp8: da's bf16 values are not stored when its consumers (the W1 weight gradient with the forward's fp8 copy
        # of h, the W1 dgrad) both run on the fp8 kernels from the epilogue's fp8 copy
        da_q8 = bool(_Q8_ONLY and _FP8["on"] and _FP8_WGRAD and hq is not None and _C.gemm8_wgrad_supported(I, H, T)
                     and ctx.needs_input_grad[0] and _fp8_dgrad_ok(w1, EPI_RES, T))
        da = gemm_dgrad(dy, w2, EPI_MUL if keep_grad else EPI_DGELU, aux=pre, dbias=g_b1.buf, dyq=dyq,
                        q8_for=w1 if ctx.needs_input_grad[0] else None, q8_only=da_q8)
        daq = _take_q8(da)
        if getattr(da, "_hsd_q8_only", False) and daq is None:
            raise RuntimeError("FFN backward: the GELU-gradient product's fp8 copy was not handed over")
        r_b1 = g_b1.done()
        r_w1 = wgrad_done(g_w1, da, h2d, daq, hq)
        dh = gemm_dgrad(da, w1, EPI_RES, aux=dz, dyq=daq) if ctx.needs_input_grad[0] else None
        return (dh.view(dout.shape) if dh is not None else None, r_w1, r_b1, r_w2, r_b2, r_lnw, r_lnb,
                None, None, None, None)


def ffn_block(h, w1, b1, w2, b2, ln_w, ln_b, eps, p, seed, q8_next=None):
    """``q8_next``: the next layer's QKV weight (its fp8 input copy is written by this block's LayerNorm)."""
    return _FFNBlock.apply(h, w1, b1, w2, b2, ln_w, ln_b, eps, p, seed, q8_next)


# ------------------------------------------------------------------------------------------ attention mask
def key_mask_bias(attention_mask):
    """[B, S] 0/1 mask -> additive fp32 bias (0 keep, float32 min masked), one kernel (ops/reference.py formula)."""
    am = attention_mask.contiguous()
    out = torch.empty(am.shape, dtype=torch.float32, device=am.device)
    _C.mask_bias(am, out)
    return out


# ------------------------------------------------------------------------------------------ classification head
_ACT = {"tanh": 0, "relu": 1}


def cls_head_ok(h, w1, w2) -> bool:
    H = h.shape[-1]
    return (h.dtype == torch.bfloat16 and h.dim() == 3 and H % 8 == 0 and H <= 1024 and 1 <= w2.shape[0] <= 4
            and w1.shape[0] == H and (h.shape[1] * H) % 8 == 0)


class _ClsHead(torch.autograd.Function):
    """First-token rows of h -> dense (gemm2, bias epilogue) -> fused act / dropout / classifier / CE / accuracy
    (cls_head.hip). Backward: one fused kernel (CE grad, classifier dgrad + fp32 dW2 / db2 into main_grad, dropout,
    act') -> dense dgrad written into the first-token rows of a zeroed dh, wgrad, bias column sums."""

    @staticmethod
    def forward(ctx, h, w1, b1, w2, b2, labels, act, p_in, seed_in, p, seed):
        B, S, H = h.shape
        C = w2.shape[0]
        x = h.reshape(B, S * H)[:, :H]  # the [CLS] rows, read in place (row stride S*H)
        if p_in > 0:
            x = dropout(x.contiguous(), p_in, seed_in)
        pre = gemm_fwd(x, w1, EPI_BIAS, bias=b1) if _nt_ok(B, H, H, EPI_BIAS) else torch.addmm(b1, x, w1.t())
        t = torch.empty_like(pre)
        logits = torch.empty((B, C), dtype=h.dtype, device=h.device)
        nblk = _C.cls_head_blocks(B)
        partials = torch.empty(nblk * 4, dtype=torch.float32, device=h.device)
        stats = torch.empty(4, dtype=torch.float32, device=h.device)
        lab = labels.contiguous().long()
        _C.cls_head_fwd(pre, w2, b2, lab, t, logits, partials, stats, _ACT[act], float(p), _s64(seed))
        ctx.save_for_backward(x, w1, b1, t, w2, b2, logits, lab, stats)
        ctx.cfg = (act, float(p_in), seed_in, float(p), seed, B, S, H)
        ctx.mark_non_differentiable(logits, stats)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the non-differentiable outputs
        return stats[0], logits, stats

    @staticmethod
    def backward(ctx, dloss, _dlogits, _dstats):
        x, w1, b1, t, w2, b2, logits, lab, stats = ctx.saved_tensors
        act, p_in, seed_in, p, seed, B, S, H = ctx.cfg
        g_w1, g_b1, g_w2, g_b2 = _Grad(w1), _Grad(b1), _Grad(w2), _Grad(b2)
        dpre = torch.empty_like(t)
        if dloss is None:
            dloss = torch.zeros((), dtype=torch.float32, device=t.device)
        dl = dloss.reshape(1).to(torch.float32).contiguous()
        _C.cls_head_bwd(t, w2, logits, lab, stats, dl, dpre, g_w2.buf, g_b2.buf, _ACT[act], p, _s64(seed))
        r_w2, r_b2 = g_w2.done(), g_b2.done()
        _C.colsum(dpre, g_b1.buf)
        r_b1 = g_b1.done()
        if _C.gemm2_supported(1, 1, 7, H, H, B):
            gemm_wgrad_(g_w1, dpre, x)
        elif B < 64:
            _C.small_wgrad(dpre, x, g_w1.buf.view(H, H))
        else:
            _wgrad_(g_w1, dpre, x)
        r_w1 = g_w1.done()
        dh = None
        if ctx.needs_input_grad[0]:
            dh = torch.empty((B, S, H), dtype=dpre.dtype, device=dpre.device)
            _C.memset0(dh)
            dst = dh.reshape(B, S * H)[:, :H]  # the [CLS] rows of dh (row stride S*H)
            if p_in > 0:
                dx = gemm_dgrad(dpre, w1) if _nt_ok(B, H, H, EPI_STORE) else torch.mm(dpre, w1)
                _C.dropout(dx, dx, p_in, _s64(seed_in))
                dst.copy_(dx)
            elif _C.gemm2_supported(0, 1, EPI_STORE, B, H, H):
                _C.gemm2(dpre, w1, dst, 0, 1, EPI_STORE, None, None, None, 0.0, 0, 0, None, None)  # reads W1 as is
            else:
                dst.copy_(torch.mm(dpre, w1))
        return dh, r_w1, r_b1, r_w2, r_b2, None, None, None, None, None, None


def cls_head(h, w1, b1, w2, b2, labels, act, p_in, seed_in, p, seed):
    """(loss, logits, stats) of the fused classification head (labels required); stats = fp32
    {mean loss, argmax hits, rows scored, loss sum}."""
    return _ClsHead.apply(h, w1, b1, w2, b2, labels, act, p_in, seed_in, p, seed)


# ------------------------------------------------------------------------------------------ masked-LM head
def mlm_head_ok(h2d, w1, wemb) -> bool:
    T, H = h2d.shape
    Vp = wemb.shape[0]
    return (H % 64 == 0 and w1.shape == (H, H) and Vp % 256 == 0 and wemb.shape[1] == H and wemb.is_contiguous()
            and _C.gemm2_supported(0, 0, EPI_BIAS, 64, Vp, H) and _C.gemm2_supported(0, 1, EPI_STORE, 64, H, Vp))


class _MlmHead(torch.autograd.Function):
    """RoBERTa LM head on the masked rows, every GEMM on gemm2 (SURVEY.md §2.10 K16 MLM variant):

    forward   x = h[masked] (row count padded to a multiple of 64 with ignored rows) -> gemm2 NT, bias + GELU
              epilogue writing pre-activation and activation -> LN kernel -> gemm2 NT against the tied word
              embeddings [Vp, H] (Vp = vocabulary padded to 256) with the lm_head bias -> xent kernel over the real
              vocabulary columns (the padding columns get zero gradient)
    backward  decoder bias grad = column sums of dlogits; tied-embedding grad += dlogitsᵀ · y (gemm2 TT: the
              padded token count is a whole number of 64-token K-tiles); dy = dlogits · Wemb (gemm2 NT reading the
              table directly as its k-strided B); LN bwd; GELU' + dense bias grad (one kernel); dense wgrad / dgrad;
              the masked rows' gradient into a zeroed dh."""

    @staticmethod
    def forward(ctx, h2d, labels, w1, b1, ln_w, ln_b, eps, wemb, bias, vocab):
        T, H = h2d.shape
        Vp = wemb.shape[0]
        lab = labels.reshape(-1)
        sel = lab.ne(-100).nonzero(as_tuple=True)[0]
        n = int(sel.numel())
        npad = max(64, -(-n // 64) * 64)
        idx = torch.zeros(npad, dtype=torch.long, device=h2d.device)
        idx[:n] = sel
        tgt = torch.full((npad,), -100, dtype=torch.long, device=h2d.device)
        tgt[:n] = lab.index_select(0, sel)
        x = h2d.index_select(0, idx)
        act = torch.empty((npad, H), dtype=h2d.dtype, device=h2d.device)
        pre = gemm_fwd(x, w1, EPI_BIAS_GELU, bias=b1, out2=act)
        y, mean, rstd = _ln_fwd(act, ln_w, ln_b, eps)
        logits = gemm_fwd(y, wemb, EPI_BIAS, bias=bias)
        stats = torch.zeros(2, dtype=torch.float32, device=h2d.device)
        n_valid = torch.full((1,), float(n), dtype=torch.float32, device=h2d.device)
        dlogits = torch.empty_like(logits)
        _C.xent(logits, tgt, dlogits, stats, n_valid, vocab)
        loss = stats[0] * (1.0 / max(n, 1))
        ctx.save_for_backward(x, sel, w1, b1, pre, act, y, mean, rstd, ln_w, ln_b, wemb, bias, dlogits)
        ctx.cfg = (T, H, n)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)
        return loss, logits[:n, :vocab], stats[1]

    @staticmethod
    def backward(ctx, dloss, _dlogits, _dcorrect):
        x, sel, w1, b1, pre, act, y, mean, rstd, ln_w, ln_b, wemb, bias, dlogits = ctx.saved_tensors
        T, H, n = ctx.cfg
        g_wemb, g_w1, g_b1, g_lnw, g_lnb, g_bias = _Grad(wemb), _Grad(w1), _Grad(b1), _Grad(ln_w), _Grad(ln_b), _Grad(bias)
        if dloss is None:
            dloss = torch.zeros((), dtype=torch.float32, device=x.device)
        dl = dloss.reshape(1).to(torch.float32)
        # decoder bias: column sums of dlogits, scaled by the incoming loss gradient
        cs = torch.zeros(dlogits.shape[1], dtype=torch.float32, device=x.device)
        _C.colsum(dlogits, cs)
        g_bias.buf.add_(cs * dl)
        # tied embedding table: += dlogitsᵀ · (y · dloss)   (dlogits is already 1/n-scaled by the CE kernel)
        gemm_wgrad_(g_wemb, dlogits, (y * dl.to(y.dtype)).contiguous())
        r_wemb = g_wemb.done()
        dy = torch.empty_like(y)
        _C.gemm2(dlogits, wemb, dy, 0, 1, EPI_STORE, None, None, None, 0.0, 0, 0, None, None)
        dy.mul_(dl.to(dy.dtype))
        dact = torch.empty_like(act)
        _C.ln_bwd(dy, act, mean, rstd, ln_w, None, dact, None, g_lnw.buf, g_lnb.buf, None, 0.0, 0)
        dpre = torch.empty_like(pre)
        _C.gelu_bwd_colsum(dact, pre, dpre, g_b1.buf)
        gemm_wgrad_(g_w1, dpre, x)
        dh = None
        if ctx.needs_input_grad[0]:
            dx = gemm_dgrad(dpre, w1)
            dh = torch.empty((T, H), dtype=dx.dtype, device=dx.device)
            _C.memset0(dh)
            dh.index_copy_(0, sel, dx[:n])
        return (dh, None, g_w1.done(), g_b1.done(), g_lnw.done(), g_lnb.done(), None, r_wemb, g_bias.done(), None)


def mlm_head(h2d, labels, w1, b1, ln_w, ln_b, eps, wemb, bias, vocab):
    """(loss, logits [n_masked, vocab], argmax hits) of the fused masked-LM head."""
    return _MlmHead.apply(h2d, labels, w1, b1, ln_w, ln_b, eps, wemb, bias, vocab)


# ------------------------------------------------------------------------------------------ loss
class _CrossEntropy(torch.autograd.Function):
    """Mean softmax cross-entropy over non-ignored rows (-100) with the gradient produced by the same
    kernel (xent.hip); also returns the argmax-correct count as a non-differentiable output."""

    @staticmethod
    def forward(ctx, logits, labels):
        lg = logits.contiguous()
        lab = labels.contiguous().long()
        n_valid = lab.ne(-100).sum().to(torch.float32).reshape(1)
        stats = torch.zeros(2, dtype=torch.float32, device=lg.device)
        dl = torch.empty_like(lg) if ctx.needs_input_grad[0] else None
        _C.xent(lg, lab, dl, stats, n_valid)
        ctx.save_for_backward(dl if dl is not None else stats)
        loss = stats[0:1] / n_valid.clamp(min=1.0)
        ctx.mark_non_differentiable(stats)
        return loss.reshape(()), stats[1]

    @staticmethod
    def backward(ctx, dloss, _dcorrect):
        (dl,) = ctx.saved_tensors
        return dl * dloss.to(dl.dtype), None


def cross_entropy(logits, labels):
    """(loss, correct_count) for [R, V] logits (bf16 / fp32) and int labels (-100 ignored)."""
    if logits.dtype not in (torch.bfloat16, torch.float32) or logits.dim() != 2:
        from .reference import accuracy_count, cross_entropy as ref

        return ref(logits, labels), accuracy_count(logits, labels)
    return _CrossEntropy.apply(logits, labels)
