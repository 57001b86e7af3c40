"""fp32 step on hand-written kernels (ops/hip32.py, csrc/kernels/fp32.hip; VERDICT r3 'missing 2'): each kernel vs a
plain fp32/fp64 torch reference of the same op, then a bert-base-shaped 2-layer training step on the GPU vs the same
step on the CPU reference ops, with a kernel trace that must hold no library GEMM / softmax / bmm kernel."""
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _h32():
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip32

    return hip32


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


@pytest.mark.parametrize("ksplit", ["auto", "1"])
@pytest.mark.parametrize("M,K,N", [(300, 768, 768), (1024, 768, 3072), (256, 3072, 768), (64, 768, 2304),
                                   (4096, 1024, 1024)])
def test_split_product_gemms(gpu, M, K, N, ksplit, monkeypatch):
    """x·wᵀ, dy·w and the weight gradient on the split-product MFMA GEMM: per element within 2^-14 of Σ|products|
    (the three-term split's bound is ~2^-15), and ~1e-6 relative overall against fp64. ksplit "auto": grids of at most
    half the CUs run as K-split fp32 slabs + one summing pass (gemm2_f32nt_splits); "1": one pass."""
    if ksplit == "1":
        monkeypatch.setenv("HSD_F32NT_SPLITS", "1")
    h = _h32()
    torch.manual_seed(M + N)
    x, w = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu) * 0.05
    y = h.mm_nt(x, w)
    ref = x.double() @ w.double().t()
    mag = x.abs().double() @ w.abs().double().t()
    assert bool(((y.double() - ref).abs() <= 2.0 ** -14 * mag + 1e-30).all())
    assert _rel(y, ref) < 1e-5
    dy = torch.randn(M, N, device=gpu)
    dx = h.mm_dgrad(dy, w)
    ref = dy.double() @ w.double()
    assert bool(((dx.double() - ref).abs() <= 2.0 ** -14 * (dy.abs().double() @ w.abs().double()) + 1e-30).all())
    from huggingface_sagemaker_tensorflow_distributed_amd.ops.hip import _Grad

    g0 = torch.randn(N, K, device=gpu)
    p = torch.nn.Parameter(torch.zeros(N, K, device=gpu))
    p.main_grad = g0.clone()
    gw = _Grad(p)
    h.wgrad_(gw, dy, x)
    ref = g0.double() + dy.double().t() @ x.double()
    mag = g0.abs().double() + dy.abs().double().t() @ x.abs().double()
    assert bool(((p.main_grad.double() - ref).abs() <= 2.0 ** -14 * mag + 1e-30).all())


def _grads(fn, *args):
    """Run fn(*args) -> scalar, backward, return (value, [grad of each arg that requires grad])."""
    out = fn(*args)
    out.backward()
    return out.detach(), [a.grad.detach().clone() for a in args if isinstance(a, torch.Tensor) and a.requires_grad]


@pytest.mark.parametrize("M,N", [(4096, 1024), (4096, 4096), (300, 36), (64, 2), (1000, 772), (3, 1028)])
def test_colsum32_accumulates_column_sums(gpu, M, N):
    """colsum32 (the fp32 bias gradients): dbias += column sums, 16-B path (N % 4 == 0) and scalar path."""
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip32

    x = torch.randn(M, N, device=gpu)
    d = torch.randn(N, device=gpu)
    want = d.double() + x.double().sum(0)
    hip32._C.colsum32(x, d)
    torch.cuda.synchronize()
    err = float((d.double() - want).abs().max())
    assert err <= 1e-5 * max(1.0, float(x.abs().sum(0).max())), err


@pytest.mark.parametrize("R,C", [(4096, 1024), (128, 772), (64, 3072)])
def test_split3_dual_matches_two_splits(gpu, R, C):
    """split3_dual (both layouts of a linear layer's incoming gradient from one read) == two split3 passes, bit for
    bit, for the 16-B (C % 8 == 0) and 8-B paths."""
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip32

    x = torch.randn(R, C, device=gpu) * 3.0
    cols = torch.empty(R, 3 * C, device=gpu, dtype=torch.bfloat16)
    rows = torch.empty(3 * R, C, device=gpu, dtype=torch.bfloat16)
    hip32._C.split3_dual(x, cols, hip32.PAT_A, rows, hip32.PAT_B)
    assert torch.equal(cols, hip32._split(x, hip32.PAT_A))
    assert torch.equal(rows, hip32._split(x, hip32.PAT_B, rows=True))
    hi, lo = cols[:, :C].float(), cols[:, 2 * C:].float()
    assert torch.equal(cols[:, :C], cols[:, C:2 * C])
    assert float((hi + lo - x).abs().max()) <= 2.0 ** -16 * float(x.abs().max())


@pytest.mark.parametrize("path", ["mfma", "valu"])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("S", [128, 512])
def test_attention32_fwd_bwd(gpu, p, S, path, monkeypatch):
    """fp32 attention forward + backward == the fp64 reference ops (same dropout masks): the split-product MFMA kernels
    (attention32m.hip, default; measured ~6e-6 / ~8e-6 relative error) and the exact-FMA vector kernels (fp32.hip)."""
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import reference as R

    monkeypatch.setattr(_h32(), "_ATTN32M", path == "mfma")

    B, heads = 2, 4
    H = heads * 64
    torch.manual_seed(S)
    qkv = torch.randn(B * S, 3 * H, device=gpu)
    am = torch.ones(B, S, device=gpu)
    am[1, S - 37:] = 0
    mb = R.key_mask_bias(am)
    g = torch.randn(B * S, H, device=gpu)
    a = qkv.clone().requires_grad_()
    out = _h32().attention(a, mb, B, S, heads, p, 1234)
    (out * g).sum().backward()
    b = qkv.clone().double().requires_grad_()
    ref = R.attention(b, mb.double(), B, S, heads, p, 1234, p > 0)  # runs in fp32 internally
    (ref * g.double()).sum().backward()
    assert _rel(out, ref) < 2e-5
    assert _rel(a.grad, b.grad) < 2e-4


def test_layernorm_embedding_dropout32(gpu):
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import reference as R

    h = _h32()
    torch.manual_seed(3)
    Bn, S, H, V = 4, 64, 768, 1000
    word = torch.randn(V, H, device=gpu) * 0.02
    pos, typ = torch.randn(512, H, device=gpu) * 0.02, torch.randn(2, H, device=gpu) * 0.02
    lw, lb = 1 + 0.1 * torch.randn(H, device=gpu), 0.1 * torch.randn(H, device=gpu)
    ids = torch.randint(0, V, (Bn, S), device=gpu)
    pids = torch.arange(S, device=gpu).expand(Bn, S)
    tids = torch.zeros_like(ids)
    g = torch.randn(Bn, S, H, device=gpu)
    ps = [t.clone().requires_grad_() for t in (word, pos, typ, lw, lb)]
    out = h.embed_ln(ids, pids, tids, *ps, 1e-12, 0.1, 99)
    (out * g).sum().backward()
    qs = [t.clone().requires_grad_() for t in (word, pos, typ, lw, lb)]
    ref = R.embed_ln(ids, pids, tids, *qs, 1e-12, 0.1, 99, True)
    (ref * g).sum().backward()
    assert _rel(out, ref) < 1e-5
    for a, b in zip(ps, qs):
        assert _rel(a.grad, b.grad) < 1e-4
    x = torch.randn(257, H, device=gpu, requires_grad=True)
    y = h.layer_norm(x, lw, lb, 1e-5)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    x2 = x.detach().clone().requires_grad_()
    y2 = torch.nn.functional.layer_norm(x2, (H,), lw, lb, 1e-5)
    (y2 * gy).sum().backward()
    assert _rel(y, y2) < 1e-6 and _rel(x.grad, x2.grad) < 1e-5


def _bert2(seed=0):
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config

    cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=2)
    return build_model(cfg, seed=seed)


def test_fp32_bert_step_on_kernels_matches_cpu(gpu):
    """A bert-base-shaped 2-layer training step (dropout on, padded batch) with --dtype fp32 semantics: the GPU step on
    the fp32 kernels reproduces the CPU fp32 reference step -- loss within 1e-4 relative, every parameter gradient
    within 1e-3 relative -- and its kernel trace holds no library GEMM (Cijk) and no ATen softmax / bmm kernel."""
    torch.manual_seed(0)
    cpu = _bert2()
    dev = copy.deepcopy(cpu).to(gpu)
    B, S = 4, 128
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1000, 30000, (B, S), generator=g)
    am = torch.ones(B, S, dtype=torch.long)
    am[2, 90:] = 0
    am[3, 40:] = 0
    labels = torch.randint(0, 2, (B,), generator=g)
    res = {}
    for name, model, d in (("cpu", cpu, "cpu"), ("gpu", dev, gpu)):
        model.train()
        model.rng.new_step(0)
        model.zero_grad(set_to_none=True)
        prof = None
        if name == "gpu":
            prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA])
            prof.__enter__()
        loss, logits = model(ids.to(d), attention_mask=am.to(d), labels=labels.to(d))
        loss.backward()
        if prof is not None:
            torch.cuda.synchronize()
            prof.__exit__(None, None, None)
            names = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
            bad = [n for n in names if "hsd::" not in n and ("Cijk" in n or "softmax" in n.lower() or "bmm" in n.lower()
                                                             or "gemm" in n.lower())]
            assert not bad, bad
            assert any("hsd::f32k::attn32" in n for n in names), sorted(names)[:40]
            assert any("gemm2_kernel" in n or "gemm2s_kernel" in n for n in names), sorted(names)[:40]
        res[name] = (float(loss), {k: p.grad.detach().float().cpu() for k, p in model.named_parameters()
                                   if p.grad is not None})
    (lc, gc), (lg, gg) = res["cpu"], res["gpu"]
    assert abs(lg - lc) <= 1e-4 * abs(lc), (lg, lc)
    assert set(gc) == set(gg)
    worst = max((_rel(gg[k], gc[k]), k) for k in gc if gc[k].norm() > 0)
    assert worst[0] < 1e-3, worst


@pytest.mark.parametrize("M,K,N", [(4096, 1024, 1024), (4096, 1024, 4096), (4096, 4096, 1024), (512, 768, 3072)])
def test_segmented_gemm_equals_concatenated_split_gemm(gpu, M, K, N):
    """gemm2_seg over the hi / lo halves == the GEMM over the three-block concatenations (split3) bit for bit: the same
    K order, tiles and K-splits, only the operand addresses differ (forward NT, dgrad with W read k-strided, TT weight
    gradient accumulating into C). The NT ones with HSD_SEG_NT_SMALL=0 (the slab kernels gemm2_f32nt also runs); the
    default 128 x 128-tile path (one K-split, a different summation order) against the fp64 product of the halves, and
    its in-place accumulate against write + add."""
    h = _h32()
    C_ = h._C
    torch.manual_seed(K + N)
    x, w, dy = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu) * 0.05, torch.randn(M, N, device=gpu)
    xh, xl = h._split2(x)
    wh, wl = h._split2(w)
    dh, dl = h._split2(dy)
    y_cat = torch.empty(M, N, device=gpu)
    C_.gemm2_f32nt(h._split(x, h.PAT_A), h._split(w, h.PAT_B), y_cat, 0)
    dx_cat = torch.empty(M, K, device=gpu)
    C_.gemm2_f32nt(h._split(dy, h.PAT_A), h._split(w, h.PAT_B, rows=True), dx_cat, 1)
    y_seg, dx_seg = torch.empty(M, N, device=gpu), torch.empty(M, K, device=gpu)
    try:
        os.environ["HSD_SEG_NT_SMALL"] = "0"
        C_.refresh_env()
        C_.gemm2_seg([xh, xh, xl], [wh, wl, wh], y_seg, 0, 0)
        C_.gemm2_seg([dh, dh, dl], [wh, wl, wh], dx_seg, 0, 1)
    finally:
        os.environ.pop("HSD_SEG_NT_SMALL", None)
        C_.refresh_env()
    assert torch.equal(y_seg, y_cat)
    assert torch.equal(dx_seg, dx_cat)
    f = lambda t: t.double()  # noqa: E731
    y_ref = f(xh) @ (f(wh) + f(wl)).t() + f(xl) @ f(wh).t()
    dx_ref = f(dh) @ (f(wh) + f(wl)) + f(dl) @ f(wh)
    for out, ref, lb in ((y_seg, y_ref, 0), (dx_seg, dx_ref, 1)):
        o = torch.empty_like(out)
        args = ([xh, xh, xl], [wh, wl, wh]) if lb == 0 else ([dh, dh, dl], [wh, wl, wh])
        C_.gemm2_seg(*args, o, 0, lb)
        assert float((o.double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max()), lb
        base = torch.randn_like(o)
        acc = base.clone()
        C_.gemm2_seg(*args, acc, 0, lb, True)
        torch.testing.assert_close(acc, base + o, rtol=1e-5, atol=1e-5)
    g0 = torch.randn(N, K, device=gpu)
    g_seg = g0.clone()
    C_.gemm2_seg([dh, dh, dl], [xh, xl, xh], g_seg, 1, 1)
    g_cat = g0.clone()
    sp = C_.gemm2_splits(N, K, 3 * M)
    ws = torch.empty(max(1, sp) * N * K, device=gpu)
    C_.gemm2(h._split(dy, h.PAT_A, rows=True), h._split(x, h.PAT_B, rows=True), g_cat, 1, 1, 7, None, None, None,
             0.0, 0, sp, ws, None, None, 0)
    assert torch.equal(g_seg, g_cat)


def test_producer_written_halves_equal_split2(gpu):
    """The bf16 halves that epi32 (bias; bias + GELU; dgrad x GELU'), dropout32 and ln32_fwd write beside (or instead
    of) their fp32 output equal split2 of that output bit for bit: the fp32 blocks feed them to the segmented GEMMs in
    place of a split2 pass."""
    h = _h32()
    C_ = h._C
    torch.manual_seed(3)
    M, N = 512, 1024
    y, b, aux = torch.randn(M, N, device=gpu), torch.randn(N, device=gpu), torch.randn(M, N, device=gpu)

    def halves(t):
        return h._split2(t.contiguous())

    for kind in (0, 1, 4):
        yk = y.clone()
        out = torch.empty_like(y)
        C_.epi32(yk, b if kind < 4 else None, aux if kind == 4 else None, out, kind, 0.0, 0)
        hi, lo = h._halves_like(y)
        yk2 = y.clone()
        C_.epi32(yk2, b if kind < 4 else None, aux if kind == 4 else None, None if kind < 2 else torch.empty_like(y),
                 kind, 0.0, 0, hi, lo)
        rh, rl = halves(out)
        assert torch.equal(hi, rh) and torch.equal(lo, rl), kind
        if kind == 1:
            assert torch.equal(yk2, yk)  # the pre-activation is still written
    out = torch.empty_like(y)
    hi, lo = h._halves_like(y)
    C_.dropout32(y, out, 0.1, 1234, hi, lo)
    ref = torch.empty_like(y)
    C_.dropout32(y, ref, 0.1, 1234)
    assert torch.equal(out, ref)
    rh, rl = halves(ref)
    assert torch.equal(hi, rh) and torch.equal(lo, rl)
    g, bb = torch.randn(N, device=gpu), torch.randn(N, device=gpu)
    out, mean, rstd = torch.empty_like(y), torch.empty(M, device=gpu), torch.empty(M, device=gpu)
    C_.ln32_fwd(y, g, bb, out, mean, rstd, 1e-12, hi, lo)
    ref = torch.empty_like(y)
    C_.ln32_fwd(y, g, bb, ref, mean, rstd, 1e-12)
    assert torch.equal(out, ref)
    rh, rl = halves(ref)
    assert torch.equal(hi, rh) and torch.equal(lo, rl)


def test_published_halves_are_taken_only_for_their_tensor(gpu):
    """The block-output halves hand-off (hip32._publish_halves / _take_halves) serves only the same, unmodified
    storage, once."""
    h = _h32()
    t = torch.randn(128, 256, device=gpu)
    hi, lo = h._split2(t)
    h._publish_halves(t, hi, lo)
    assert h._take_halves(torch.randn(128, 256, device=gpu)) is None
    t.add_(1.0)
    assert h._take_halves(t) is None  # modified in place since
    h._publish_halves(t, hi, lo)
    got = h._take_halves(t.view(128, 256))
    assert got is not None and got[0].data_ptr() == hi.data_ptr()
    assert h._take_halves(t) is None  # taken once


def test_adam_writes_weight_halves_and_stale_halves_are_resplit(gpu):
    """fp32 store: the fused Adam writes every updated weight's bf16 hi / lo halves (= split2 of the new master) in the
    same pass, and a weight changed in place outside the optimizer is split again at use (weight_split)."""
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    h = _h32()
    model = _bert2().to(gpu)
    store = FlatParamStore(model, gpu, compute_dtype=torch.float32)
    assert store.split_hi is not None and store.splits_current()
    opt = FusedAdam(store, lr=1e-3)
    store.grad.normal_()
    opt.step()
    hi, lo = h._split2(store.master)
    assert torch.equal(store.split_hi, hi) and torch.equal(store.split_lo, lo)
    w = model.encoder.layers[0].qkv_weight
    wh, wl = h.weight_split(w)
    assert wh.data_ptr() == w._hsd_split[0].data_ptr()  # the store's halves, no split at use
    with torch.no_grad():
        w.mul_(2.0)
    wh2, wl2 = h.weight_split(w)
    assert wh2.data_ptr() != w._hsd_split[0].data_ptr()
    rh, rl = h._split2(w.detach().contiguous())
    assert torch.equal(wh2, rh) and torch.equal(wl2, rl)


def test_fused_fp32_blocks_match_unfused_ops(gpu):
    """_AttnBlock32 / _FFNBlock32 (the block's first dgrad accumulated in place into the residual gradient) == the
    unfused fp32 ops (linear, attention, dense_residual_ln: autograd adds the two gradients of h): outputs, the input
    gradient and the weight gradients bit for bit (the same kernels in the same order; the residual add is the one
    commutative fp32 add); bias / LayerNorm gradients to fp32 atomic-order rounding."""
    h32 = _h32()
    torch.manual_seed(5)
    B, S, H, heads, inner = 2, 512, 1024, 16, 4096
    h0 = torch.randn(B * S, H, device=gpu)
    mk = lambda *s: (torch.randn(*s, device=gpu) * 0.03).requires_grad_()  # noqa: E731
    qkv_w, qkv_b, out_w, out_b = mk(3 * H, H), mk(3 * H), mk(H, H), mk(H)
    w1, b1, w2, b2 = mk(inner, H), mk(inner), mk(H, inner), mk(H)
    ln = [(1 + 0.1 * torch.randn(H, device=gpu)).requires_grad_() for _ in range(2)]
    lb = [(0.1 * torch.randn(H, device=gpu)).requires_grad_() for _ in range(2)]
    am = torch.ones(B, S, dtype=torch.long, device=gpu)
    am[1, 300:] = 0
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import reference as ref

    mb = ref.key_mask_bias(am)
    params = [qkv_w, qkv_b, out_w, out_b, w1, b1, w2, b2] + ln + lb
    assert h32.attn_block_ok(h0, qkv_w, S, heads) and h32.ffn_block_ok(h0, w1)
    d = torch.randn(B * S, H, device=gpu)
    res = []
    for fused in (True, False):
        h = h0.clone().requires_grad_()
        for p in params:
            p.grad = None
        if fused:
            x = h32.attn_block(h, qkv_w, qkv_b, out_w, out_b, ln[0], lb[0], 1e-12, mb, B, S, heads, 0.1, 11, 0.1, 12)
            y = h32.ffn_block(x, w1, b1, w2, b2, ln[1], lb[1], 1e-12, 0.1, 13)
        else:
            qkv = h32.linear(h, qkv_w, qkv_b)
            ctx = h32.attention(qkv, mb, B, S, heads, 0.1, 11)
            x = h32.dense_residual_ln(ctx, out_w, out_b, h, ln[0], lb[0], 1e-12, 0.1, 12)
            a = h32.linear_gelu(x, w1, b1)
            y = h32.dense_residual_ln(a, w2, b2, x, ln[1], lb[1], 1e-12, 0.1, 13)
        y.backward(d)
        res.append((y.detach().clone(), h.grad.clone(), [p.grad.clone() for p in params]))
    (y0, g0, p0), (y1, g1, p1) = res
    assert torch.equal(y0, y1)
    assert torch.equal(g0, g1)
    for a, b in zip(p0, p1):
        if a.dim() == 2:
            assert torch.equal(a, b)  # weight gradients: the same GEMMs
        else:  # bias / LayerNorm gradients: fp32 column-sum atomics, summation order differs run to run
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * float(b.abs().max()))
