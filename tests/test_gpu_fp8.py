"""fp8 path (csrc/kernels/fp8.hip, gemm8.hip) vs plain-PyTorch fp32 references.

The quantised operands are dequantised with torch's own OCP float8 dtypes (float8_e4m3fn / float8_e5m2),
which also pins the encoding the gfx950 conversion instructions produce (OCP, not the MI300 fnuz one).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip

    return hip


def _deq(q, sinv, fmt):
    dt = torch.float8_e4m3fn if fmt == 0 else torch.float8_e5m2
    return q.view(dt).float() * sinv.float()


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("n", [4096 * 33, 1000 * 7 + 3])
def test_fp8_quant_roundtrip(gpu, fmt, n):
    hip = _hip()
    torch.manual_seed(0)
    x = (torch.randn(n, device=gpu) * 3).bfloat16()
    q, sinv = hip.quant_fp8(x, fmt)
    amax = x.float().abs().max()
    fmax = 448.0 if fmt == 0 else 57344.0
    torch.testing.assert_close(sinv, (amax / fmax).reshape(1), rtol=1e-6, atol=0)
    d = _deq(q, sinv, fmt)
    rel = 2.0 ** -4 if fmt == 0 else 2.0 ** -3  # half an ulp of a 3 / 2-bit mantissa
    err = (d - x.float()).abs()
    tol = rel * x.float().abs() + 2.0 ** -9 * amax / fmax * 64  # subnormal floor
    assert (err <= tol).all(), float(err.max())
    # the largest magnitude maps to the format maximum
    assert float(_deq(q, torch.ones(1, device=gpu), fmt).abs().max()) == fmax


@pytest.mark.parametrize("M,N,K,epi", [(512, 768, 768, 1), (300, 1024, 1024, 0), (1024, 3072, 768, 8),
                                       (512, 768, 3072, 3), (768, 1024, 4096, 4), (512, 768, 3072, 9),
                                       # several rounds of the persistent kernel's tiles, M edges, BN 256 and 192
                                       (32768, 1024, 1024, 4), (8292, 4096, 1024, 9), (20000, 3072, 1024, 1),
                                       (4096, 1024, 4096, 3), (16384, 4096, 1024, 8)])
@pytest.mark.parametrize("fa", [0, 1])
def test_gemm8_matches_fp32_reference(gpu, M, N, K, epi, fa):
    """The persistent fp8 kernel (gemm8pk) vs the fp32 product of the dequantised operands, every epilogue kind."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(1)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = (torch.randn(N, K, device=gpu) * 0.05).bfloat16()
    qx, sx = hip.quant_fp8(x, fa)
    qw, sw = hip.quant_fp8(w, 0)
    acc = _deq(qx, sx, fa) @ _deq(qw, sw, 0).t()
    bias = (torch.randn(N, device=gpu) * 0.1).bfloat16()
    aux = torch.randn(M, N, device=gpu).bfloat16()
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    y2 = torch.empty_like(y)
    dbias = torch.zeros(N, device=gpu) if epi == 9 else None
    C.gemm8(qx, fa, sx, qw, 0, sw, y, epi, bias if epi in (1, 2, 3, 8) else None,
            aux if epi in (3, 4, 5, 9) else None, y2 if epi in (2, 8) else None, 0.0, 0, dbias)
    if epi == 0:
        ref = acc
    elif epi == 1:
        ref = acc + bias.float()
    elif epi == 8:  # C = gelu'(y), C2 = gelu(y)
        z = (acc + bias.float()).bfloat16().float().requires_grad_()
        g = torch.nn.functional.gelu(z)
        (dg,) = torch.autograd.grad(g.sum(), z)
        torch.testing.assert_close(y2.float(), g.detach(), atol=3e-2, rtol=3e-2)
        ref = dg
    elif epi == 3:  # dropout p=0: y + bias + residual
        ref = (acc + bias.float()).bfloat16().float() + aux.float()
    elif epi == 4:
        ref = acc.bfloat16().float() + aux.float()
    else:  # 9: C = acc * aux, dbias = column sums
        ref = acc.bfloat16().float() * aux.float()
        torch.testing.assert_close(dbias, y.float().sum(0), atol=1e-1, rtol=2e-2)
    err = (y.float() - ref).abs()
    tol = 2e-2 * ref.abs().max() + 1e-2 * ref.abs()
    assert (err <= tol).float().mean() > 0.999, float(err.max())


def test_store_fp8_weight_copies(gpu):
    """FlatParamStore(fp8=True) keeps W8 / W8ᵀ in step with the bf16 weights (shared scale)."""
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    cfg = resolve_config("roberta-large").replace(num_hidden_layers=1)
    m = build_model(cfg, task="masked-lm", seed=0).to(gpu)
    store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, fp8=True)
    for name in ("qkv_weight", "attn_out_weight", "ffn1_weight", "ffn2_weight"):
        w = dict(m.named_parameters())[f"encoder.layers.0.{name}"]
        d = _deq(w._hsd_q, w._hsd_qs, 0)
        dt = _deq(w._hsd_qt, w._hsd_qs, 0)
        torch.testing.assert_close(dt, d.t(), atol=0, rtol=0)
        err = (d - w.float()).abs()
        assert (err <= 2.0 ** -4 * w.float().abs() + 1e-6).float().mean() > 0.999, name
    # after an update the copies follow
    with torch.no_grad():
        store.master.mul_(1.5)
    store.sync_compute_from_master()
    w = dict(m.named_parameters())["encoder.layers.0.ffn1_weight"]
    d = _deq(w._hsd_q, w._hsd_qs, 0)
    assert ((d - w.float()).abs() <= 2.0 ** -4 * w.float().abs() + 1e-6).float().mean() > 0.999


def test_fp8_mlm_step_tracks_bf16(gpu):
    """roberta-large (2 layers) MLM train step with fp8 GEMMs vs the same step in bf16."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    hip = _hip()
    cfg = resolve_config("roberta-large").replace(num_hidden_layers=2)
    ds = hdata.synthetic_mlm(4, 256, cfg.vocab_size, seed=3)
    ids = torch.from_numpy(ds.input_ids).long().to(gpu)
    am = torch.from_numpy(ds.attention_mask).long().to(gpu)
    labels = torch.from_numpy(ds.labels).long().to(gpu)
    out = {}
    for fp8 in (False, True):
        m = build_model(cfg, task="masked-lm", seed=0).to(gpu)
        store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, fp8=fp8)
        hip.set_fp8(fp8)
        try:
            m.train()
            m.rng.new_step(0)
            store.zero_grad()
            loss, _ = m(ids, attention_mask=am, labels=labels)
            loss.backward()
            torch.cuda.synchronize()
        finally:
            hip.set_fp8(False)
        out[fp8] = (float(loss), store.grad.float().clone())
    (l0, g0), (l1, g1) = out[False], out[True]
    assert abs(l1 - l0) / abs(l0) < 2e-2, (l0, l1)
    cos = torch.nn.functional.cosine_similarity(g0, g1, dim=0)
    assert torch.isfinite(g1).all() and cos > 0.97, float(cos)


def test_fp8_delayed_scaling_site(gpu):
    """A delayed-scaling site: the first use calibrates (amax pass), later uses scale with the previous
    step's amax (values beyond it saturate) and record the running amax for the next roll."""
    hip = _hip()
    torch.manual_seed(2)
    x = torch.randn(8192, device=gpu).bfloat16()
    a = float(x.float().abs().max())
    st = torch.zeros(2, device=gpu)
    q, sinv = hip.quant_fp8(x, 0, st)
    torch.testing.assert_close(st.cpu(), torch.tensor([a, a]), rtol=0, atol=0)
    torch.testing.assert_close(sinv.cpu(), torch.tensor([a / 448.0]), rtol=1e-6, atol=0)
    # roll (what FlatParamStore.refresh_fp8 does), then a tensor twice as large
    st[0] = st[1]
    st[1] = 0
    q2, sinv2 = hip.quant_fp8(x * 2, 0, st)
    torch.testing.assert_close(sinv2.cpu(), torch.tensor([a / 448.0]), rtol=1e-6, atol=0)
    assert abs(float(st[1]) - 2 * a) <= 1e-6 * a
    d = _deq(q2, sinv2, 0)
    assert float(d.abs().max()) <= a * (1 + 1e-6)  # saturated at the old amax


@pytest.mark.parametrize("rows,H", [(4096, 768), (1000, 1024), (333, 512)])
def test_ln_fwd_q8_equals_ln_then_quant(gpu, rows, H):
    """LN forward writing the output's fp8 copy (delayed-scaling site) == LN, then the standalone quantiser with the
    same site: identical bf16 output, fp8 bytes, sinv and tracked amax."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(3)
    z = (torch.randn(rows, H, device=gpu) * 2 + 0.3).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    b = (0.1 * torch.randn(H, device=gpu)).bfloat16()
    out_ref, mean_ref, rstd_ref = (torch.empty_like(z), torch.empty(rows, device=gpu), torch.empty(rows, device=gpu))
    C.ln_fwd(z, None, w, b, None, out_ref, mean_ref, rstd_ref, 1e-12, 0.0, 0)
    st_ref = torch.tensor([3.0, 0.0], device=gpu)
    st_ref._hsd_cal = True
    q_ref, s_ref = hip.quant_fp8(out_ref, 0, st_ref)
    st = torch.tensor([3.0, 0.0], device=gpu)
    out, mean, rstd = torch.empty_like(z), torch.empty(rows, device=gpu), torch.empty(rows, device=gpu)
    q = torch.empty(rows, H, dtype=torch.uint8, device=gpu)
    sinv = torch.empty(1, device=gpu)
    C.ln_fwd_q8(z, w, b, out, mean, rstd, 1e-12, q, st[0:1], sinv, st[1:2])
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref) and torch.equal(mean, mean_ref) and torch.equal(rstd, rstd_ref)
    assert torch.equal(q, q_ref)
    assert torch.equal(sinv, s_ref) and torch.equal(st, st_ref)


@pytest.mark.parametrize("rows,H,p,fmt", [(4096, 768, 0.1, 0), (1000, 1024, 0.0, 1), (2048, 1024, 0.1, 1)])
def test_ln_bwd_q8_equals_ln_bwd_then_quant(gpu, rows, H, p, fmt):
    """LN backward writing dy's fp8 copy == LN backward, then the standalone quantiser: identical dz / dy / dgamma /
    dbeta / dbias inputs to the GEMMs, fp8 bytes, sinv and tracked amax."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(4)
    z = torch.randn(rows, H, device=gpu).bfloat16()
    dout = torch.randn(rows, H, device=gpu).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    mean = z.float().mean(1)
    rstd = torch.rsqrt(z.float().var(1, unbiased=False) + 1e-12)
    res = {}
    for fused in (False, True):
        dz = torch.empty_like(z) if p > 0 else None
        dy = torch.empty_like(z)
        dg, db, dbias = (torch.zeros(H, device=gpu) for _ in range(3))
        st = torch.tensor([5.0, 0.0], device=gpu)
        if fused:
            q = torch.empty(rows, H, dtype=torch.uint8, device=gpu)
            sinv = torch.empty(1, device=gpu)
            C.ln_bwd_q8(dout, z, mean, rstd, w, dz, dy, dg, db, dbias, p, 11, q, st[0:1], sinv, st[1:2], fmt)
        else:
            C.ln_bwd(dout, z, mean, rstd, w, dz, dy, None, dg, db, dbias, p, 11)
            st._hsd_cal = True
            q, sinv = hip.quant_fp8(dy, fmt, st)
        torch.cuda.synchronize()
        res[fused] = (dz, dy, dg, db, dbias, q, sinv, st)
    a, b = res[False], res[True]
    for i, (x, y) in enumerate(zip(a, b)):
        if x is None:
            assert y is None
        elif i in (2, 3, 4):  # column sums: fp32 atomics in a different order
            torch.testing.assert_close(y, x, rtol=1e-5, atol=1e-4)
        else:
            assert torch.equal(x, y), i


@pytest.mark.parametrize("rows,H,fmt", [(4096, 768, 0), (2048, 1024, 1)])
def test_ln_bwd_q8_only_skips_dy(gpu, rows, H, fmt):
    """LN backward with q8_only (dropout on): dy's bf16 buffer is left untouched, every other output (dz, the fp8 copy,
    its scale and amax, dgamma / dbeta / the bias gradient summed from the rounded dy) as when dy is stored."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(7)
    z = torch.randn(rows, H, device=gpu).bfloat16()
    dout = torch.randn(rows, H, device=gpu).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    mean = z.float().mean(1)
    rstd = torch.rsqrt(z.float().var(1, unbiased=False) + 1e-12)
    res = {}
    for only in (False, True):
        dz = torch.empty_like(z)
        dy = torch.full_like(z, 3.0)
        dg, db, dbias = (torch.zeros(H, device=gpu) for _ in range(3))
        st = torch.tensor([5.0, 0.0], device=gpu)
        q = torch.empty(rows, H, dtype=torch.uint8, device=gpu)
        sinv = torch.empty(1, device=gpu)
        C.ln_bwd_q8(dout, z, mean, rstd, w, dz, dy, dg, db, dbias, 0.1, 11, q, st[0:1], sinv, st[1:2], fmt,
                    q8_only=only)
        torch.cuda.synchronize()
        res[only] = (dz, dy, dg, db, dbias, q, sinv, st)
    a, b = res[False], res[True]
    assert bool((b[1] == 3.0).all()) and not bool((a[1] == 3.0).all())
    for i in (0, 5, 6, 7):
        assert torch.equal(a[i], b[i]), i
    for i in (2, 3, 4):
        torch.testing.assert_close(b[i], a[i], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,S,H,p", [(32, 128, 768, 0.1), (8, 512, 1024, 0.0)])
def test_embed_fwd_q8_equals_embed_then_quant(gpu, B, S, H, p):
    """The embedding forward (gather + LayerNorm + dropout) writing its output's fp8 copy == the same kernel, then the
    standalone quantiser with the same delayed-scaling site: identical bf16 output, fp8 bytes, sinv and tracked amax."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(5)
    V = 1000
    word = (torch.randn(V, H, device=gpu) * 0.05).bfloat16()
    pos = (torch.randn(S, H, device=gpu) * 0.05).bfloat16()
    typ = (torch.randn(2, H, device=gpu) * 0.05).bfloat16()
    w = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16()
    b = (0.1 * torch.randn(H, device=gpu)).bfloat16()
    ids = torch.randint(0, V, (B, S), device=gpu)
    pids = torch.arange(S, device=gpu).expand(B, S).contiguous()
    tids = torch.zeros_like(ids)
    res = {}
    for fused in (False, True):
        out = torch.empty(B * S, H, device=gpu, dtype=torch.bfloat16)
        mean, rstd = torch.empty(B * S, device=gpu), torch.empty(B * S, device=gpu)
        st = torch.tensor([2.0, 0.0], device=gpu)
        if fused:
            q = torch.empty(B * S, H, dtype=torch.uint8, device=gpu)
            sinv = torch.empty(1, device=gpu)
            C.embed_fwd(ids, pids, tids, word, pos, typ, w, b, out, mean, rstd, 1e-12, p, 21, q, st[0:1], sinv, st[1:2])
        else:
            C.embed_fwd(ids, pids, tids, word, pos, typ, w, b, out, mean, rstd, 1e-12, p, 21)
            st._hsd_cal = True
            q, sinv = hip.quant_fp8(out, 0, st)
        torch.cuda.synchronize()
        res[fused] = (out, mean, rstd, q, sinv, st)
    for i, (x, y) in enumerate(zip(res[False], res[True])):
        assert torch.equal(x, y), i


def test_fp8_fused_ln_quant_in_the_step(gpu):
    """bert-base (2 layers, S = 256) fp8 step: after calibration every fp8 GEMM operand comes from its producer (the
    embedding, the LayerNorms forward and backward, attention, the FFN epilogues): the calibrated step runs no
    standalone activation / gradient quantiser, and its gradient tracks the previous step's."""
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    hip = _hip()
    cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=2, hidden_dropout_prob=0.0,
                                                      attention_probs_dropout_prob=0.0)
    g = torch.Generator().manual_seed(0)
    # S = 256: the streaming attention kernels write their fp8 copies too (the S = 128 kernels do not: there the
    # context and dqkv would add 2 standalone quantisations per layer)
    ids = torch.randint(1000, 30000, (32, 256), generator=g).to(gpu)
    am = torch.ones(32, 256, dtype=torch.long, device=gpu)
    labels = torch.randint(0, 2, (32,), generator=g).to(gpu)
    m = build_model(cfg, seed=0).to(gpu)
    store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, fp8=True)
    hip.set_fp8(True)
    calls = {"ln_fwd_q8": 0, "ln_bwd_q8": 0, "fp8_quant": 0, "embed_fwd": 0, "gemm8_wgrad": 0}
    orig = {k: getattr(hip._C, k) for k in calls}

    class _Count:
        def __getattr__(self, k):
            f = getattr(orig_C, k)
            if k in calls:
                def w(*a, **kw):
                    calls[k] += 1
                    return f(*a, **kw)
                return w
            return f

    orig_C = hip._C
    try:
        grads = []
        for step in range(3):
            if step == 2:
                hip._C = _Count()
            m.train()
            m.rng.new_step(0)
            store.zero_grad()
            loss, _ = m(ids, attention_mask=am, labels=labels)
            loss.backward()
            torch.cuda.synchronize()
            grads.append((float(loss), store.grad.clone()))
            store.refresh_fp8()
    finally:
        hip._C = orig_C
        hip.set_fp8(False)
    # per layer: the attention block's LN writes W1's copy (+ the first FFN LN writes layer 2's QKV copy);
    # every block's LN backward writes dy's copy
    assert calls["ln_fwd_q8"] == 3 and calls["ln_bwd_q8"] == 4, calls
    # ... and the embedding writes the first layer's: a calibrated step runs no standalone activation quantiser
    assert calls["embed_fwd"] == 1 and calls["fp8_quant"] == 0, calls
    # ... and every encoder weight gradient (4 per layer) runs on the fp8 TT kernel from those same copies
    assert calls["gemm8_wgrad"] == 8, calls
    assert torch.isfinite(grads[-1][1]).all()
    cos = torch.nn.functional.cosine_similarity(grads[1][1], grads[2][1], dim=0)
    assert cos > 0.999, float(cos)


@pytest.mark.parametrize("S,p,fmt,use_km", [(512, 0.1, 0, False), (256, 0.0, 1, False), (512, 0.1, 0, True),
                                            (384, 0.1, 1, True)])
def test_attention_q8_equals_attention_then_quant(gpu, S, p, fmt, use_km):
    """Streaming attention writing the fp8 copy of its output (forward) / of dqkv (backward) == the bf16 kernels,
    then the standalone quantiser with the same delayed-scaling site (use_km: both with the forward's keep bits)."""
    hip = _hip()
    C = hip._C
    assert C.attn_q8_supported(S) and not C.attn_q8_supported(128)
    torch.manual_seed(5)
    B, heads = 2, 16
    H = heads * 64
    qkv = (torch.randn(B * S, 3 * H, device=gpu) * 0.5).bfloat16()
    mb = torch.zeros(B, S, device=gpu)
    mb[1, S - 37:] = -10000.0
    res = {}
    for fused in (False, True):
        km = hip._keep_mask(B, S, heads, p, gpu) if use_km else None
        assert (km is not None) == use_km
        out = torch.empty(B * S, H, device=gpu, dtype=torch.bfloat16)
        lse = torch.empty(B * heads * S, device=gpu)
        st = torch.tensor([2.0, 0.0], device=gpu)
        if fused:
            q, sinv = torch.empty(B * S, H, dtype=torch.uint8, device=gpu), torch.empty(1, device=gpu)
            C.attn_fwd_q8(qkv, mb, out, lse, B, S, heads, p, 9, q, st[0:1], sinv, st[1:2], km)
        else:
            C.attn_fwd(qkv, mb, out, lse, B, S, heads, p, 9, km)
            st._hsd_cal = True
            q, sinv = hip.quant_fp8(out, 0, st)
        dout = torch.randn_like(out)
        dqkv = torch.empty_like(qkv)
        ws = hip._attn_ws(B, S, heads, gpu)
        db = torch.zeros(3 * H, device=gpu)
        gst = torch.tensor([3.0, 0.0], device=gpu)
        torch.manual_seed(6)
        dout = torch.randn_like(out)
        if fused:
            gq, gs = torch.empty(B * S, 3 * H, dtype=torch.uint8, device=gpu), torch.empty(1, device=gpu)
            C.attn_bwd_q8(qkv, mb, out, dout, lse, dqkv, ws, B, S, heads, p, 9, db, gq, gst[0:1], gs, gst[1:2], fmt,
                          km)
        else:
            C.attn_bwd(qkv, mb, out, dout, lse, dqkv, ws, B, S, heads, p, 9, db, km)
            gst._hsd_cal = True
            gq, gs = hip.quant_fp8(dqkv, fmt, gst)
        torch.cuda.synchronize()
        res[fused] = (out, lse, q, sinv, st, dqkv, gq, gs, gst, db)
    a, b = res[False], res[True]
    for i, (x, y) in enumerate(zip(a, b)):
        if i == 9:
            torch.testing.assert_close(y, x, rtol=1e-5, atol=1e-4)
        else:
            assert torch.equal(x, y), i


@pytest.mark.parametrize("S,fmt", [(512, 0), (384, 1)])
def test_attention_bwd_q8_only_skips_dqkv(gpu, S, fmt):
    """Streaming attention backward with q8_only: dqkv's bf16 buffer untouched, its fp8 copy, scale, amax and the
    fused QKV bias gradient as when dqkv is stored."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(15)
    B, heads = 2, 16
    H = heads * 64
    qkv = (torch.randn(B * S, 3 * H, device=gpu) * 0.5).bfloat16()
    mb = torch.zeros(B, S, device=gpu)
    mb[1, S - 37:] = -10000.0
    out = torch.empty(B * S, H, device=gpu, dtype=torch.bfloat16)
    lse = torch.empty(B * heads * S, device=gpu)
    C.attn_fwd(qkv, mb, out, lse, B, S, heads, 0.1, 9)
    dout = torch.randn_like(out)
    res = {}
    for only in (False, True):
        dqkv = torch.full_like(qkv, 3.0)
        ws = hip._attn_ws(B, S, heads, gpu)
        db = torch.zeros(3 * H, device=gpu)
        gst = torch.tensor([3.0, 0.0], device=gpu)
        gq, gs = torch.empty(B * S, 3 * H, dtype=torch.uint8, device=gpu), torch.empty(1, device=gpu)
        C.attn_bwd_q8(qkv, mb, out, dout, lse, dqkv, ws, B, S, heads, 0.1, 9, db, gq, gst[0:1], gs, gst[1:2], fmt,
                      q8_only=only)
        torch.cuda.synchronize()
        res[only] = (dqkv, gq, gs, gst, db)
    a, b = res[False], res[True]
    assert bool((b[0] == 3.0).all()) and not bool((a[0] == 3.0).all())
    for i in (1, 2, 3):
        assert torch.equal(a[i], b[i]), i
    torch.testing.assert_close(b[4], a[4], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,N,K,epi,fmt", [(8192, 4096, 1024, 8, 0), (8192, 1024, 4096, 9, 1), (5000, 3072, 768, 9, 0)])
def test_gemm8_epilogue_q8_equals_gemm8_then_quant(gpu, M, N, K, epi, fmt):
    """The fp8 GEMM's epilogue writing the fp8 copy of its output (GELU output for the FFN1 forward, the GELU'-product
    for the FFN2 dgrad) == the same GEMM, then the standalone quantiser on the same site."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(8)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = (torch.randn(N, K, device=gpu) * 0.05).bfloat16()
    qx, sx = hip.quant_fp8(x, 0)
    qw, sw = hip.quant_fp8(w, 0)
    bias = (torch.randn(N, device=gpu) * 0.1).bfloat16()
    aux = torch.randn(M, N, device=gpu).bfloat16()
    res = {}
    for fused in (False, True):
        y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        y2 = torch.empty_like(y) if epi == 8 else None
        db = torch.zeros(N, device=gpu) if epi == 9 else None
        st = torch.tensor([1.5, 0.0], device=gpu)
        kw = {}
        if fused:
            q, sinv = torch.empty(M, N, dtype=torch.uint8, device=gpu), torch.empty(1, device=gpu)
            kw = dict(q8=q, q8_amax=st[0:1], q8_sinv=sinv, q8_track=st[1:2], q8fmt=fmt)
        C.gemm8(qx, 0, sx, qw, 0, sw, y, epi, bias if epi == 8 else None, aux if epi == 9 else None, y2, 0.0, 0, db,
                **kw)
        if not fused:
            st._hsd_cal = True
            q, sinv = hip.quant_fp8(y2 if epi == 8 else y, fmt, st)
        torch.cuda.synchronize()
        res[fused] = (y, y2, q, sinv, st, db)
    a, b = res[False], res[True]
    assert torch.equal(a[0], b[0])
    if a[1] is not None:
        assert torch.equal(a[1], b[1])
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])
    if a[5] is not None:
        torch.testing.assert_close(b[5], a[5], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,N,K,epi,fmt", [(8192, 4096, 1024, 8, 0), (8192, 1024, 4096, 9, 1)])
def test_gemm8_epilogue_q8_only_skips_the_bf16_twin(gpu, M, N, K, epi, fmt):
    """q8_only: the fp8 epilogue does not store the bf16 output its fp8 copy duplicates (C2 of the GELU epilogue, C of
    the GELU'-product one); every other output (the fp8 copy, its scale / amax, GELU', the bias-gradient column sums)
    is bit-identical to the epilogue that stores both, and the skipped buffer keeps its previous contents."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(9)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = (torch.randn(N, K, device=gpu) * 0.05).bfloat16()
    qx, sx = hip.quant_fp8(x, 0)
    qw, sw = hip.quant_fp8(w, 0)
    bias = (torch.randn(N, device=gpu) * 0.1).bfloat16()
    aux = torch.randn(M, N, device=gpu).bfloat16()
    res = {}
    for only in (False, True):
        y = torch.full((M, N), 7.0, device=gpu, dtype=torch.bfloat16)
        y2 = torch.full_like(y, 7.0) if epi == 8 else None
        db = torch.zeros(N, device=gpu) if epi == 9 else None
        st = torch.tensor([1.5, 0.0], device=gpu)
        q, sinv = torch.empty(M, N, dtype=torch.uint8, device=gpu), torch.empty(1, device=gpu)
        C.gemm8(qx, 0, sx, qw, 0, sw, y, epi, bias if epi == 8 else None, aux if epi == 9 else None, y2, 0.0, 0, db,
                q8=q, q8_amax=st[0:1], q8_sinv=sinv, q8_track=st[1:2], q8fmt=fmt, q8_only=only)
        torch.cuda.synchronize()
        res[only] = (y, y2, q, sinv, st, db)
    a, b = res[False], res[True]
    assert torch.equal(a[2], b[2]) and torch.equal(a[3], b[3]) and torch.equal(a[4], b[4])
    skipped = b[1] if epi == 8 else b[0]
    assert bool((skipped == 7.0).all())
    if epi == 8:
        assert torch.equal(a[0], b[0])  # GELU' is still stored
    else:
        torch.testing.assert_close(b[5], a[5], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("drop", [0.0, 0.1])
def test_fp8_step_q8_only_equals_writing_both(gpu, drop):
    """roberta-large (2 layers) MLM, calibrated fp8 step with fp8 weight gradients: skipping the bf16 twins of the fp8
    copies (hip._Q8_ONLY: the FFN epilogues; with dropout also the LayerNorm backwards' dy) leaves the loss and every
    gradient as with both written (the bias gradients' column atomics aside, which sum in a run-dependent order)."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    hip = _hip()
    cfg = resolve_config("roberta-large").replace(num_hidden_layers=2, hidden_dropout_prob=drop,
                                                  attention_probs_dropout_prob=drop)
    ds = hdata.synthetic_mlm(8, 256, cfg.vocab_size, seed=4)
    ids = torch.from_numpy(ds.input_ids).long().to(gpu)
    am = torch.from_numpy(ds.attention_mask).long().to(gpu)
    labels = torch.from_numpy(ds.labels).long().to(gpu)
    m = build_model(cfg, task="masked-lm", seed=0).to(gpu)
    store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, fp8=True)
    hip.set_fp8(True)
    prev = hip._Q8_ONLY
    out = {}
    try:
        for step, only in enumerate((False, False, False, True)):
            hip._Q8_ONLY = only
            n0 = hip.WGRAD8_CALLS[0]
            m.train()
            m.rng.new_step(0)
            store.zero_grad()
            loss, _ = m(ids, attention_mask=am, labels=labels)
            loss.backward()
            torch.cuda.synchronize()
            out[only] = (float(loss), store.grad.float().clone())
            if step < 2:
                store.refresh_fp8()
            if only:
                assert hip.WGRAD8_CALLS[0] - n0 == 8
    finally:
        hip._Q8_ONLY = prev
        hip.set_fp8(False)
    (l0, g0), (l1, g1) = out[False], out[True]
    assert abs(l0 - l1) <= 1e-6 * abs(l0)  # the MLM loss sums by atomics
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("M,N,T", [(768, 256, 384), (2304, 768, 4096), (512, 1024, 1152), (1024, 4096, 2048)])
@pytest.mark.parametrize("fdy", [0, 1])
def test_gemm8_wgrad_matches_dequantised_fp32(gpu, M, N, T, fdy):
    """fp8 TT weight gradient (gemm2.hip gemm8tt_kernel + slab reduce): C += dequant(dy8)ᵀ · dequant(x8), both
    operands read as the producers write them ([T][M], [T][N]); fp32 reference of the same dequantised values."""
    hip = _hip()
    torch.manual_seed(5)
    dy = (torch.randn(T, M, device=gpu) * 0.01).bfloat16()
    x = torch.randn(T, N, device=gpu).bfloat16()
    qd, sd = hip.quant_fp8(dy, fdy)
    qx, sx = hip.quant_fp8(x, 0)
    c0 = torch.randn(M, N, device=gpu)
    ref = c0.double() + _deq(qd, sd, fdy).double().t() @ _deq(qx, sx, 0).double()
    for splits in (0, 1, 3):
        c = c0.clone()
        ws = torch.empty(hip._C.gemm8_wgrad_ws_numel(M, N, T, splits), device=gpu)
        hip._C.gemm8_wgrad(0, qd, fdy, sd, qx, 0, sx, c, splits, ws)
        torch.cuda.synchronize()
        err = (c.double() - ref).abs()
        scale = (_deq(qd, sd, fdy).double().abs().t() @ _deq(qx, sx, 0).double().abs()) + c0.double().abs()
        assert (err <= 1e-5 * scale + 1e-7).all(), (splits, float((err / (scale + 1e-12)).max()))


def test_fp8_wgrad_step_tracks_bf16_wgrad(gpu):
    """roberta-large (2 layers) MLM, calibrated fp8 step: weight gradients on the fp8 TT kernel vs the same step with
    bf16 weight gradients (HSD_FP8_WGRAD=0) from the same fp8 forward / dgrad."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore

    hip = _hip()
    cfg = resolve_config("roberta-large").replace(num_hidden_layers=2, hidden_dropout_prob=0.0,
                                                  attention_probs_dropout_prob=0.0)
    ds = hdata.synthetic_mlm(8, 256, cfg.vocab_size, seed=3)
    ids = torch.from_numpy(ds.input_ids).long().to(gpu)
    am = torch.from_numpy(ds.attention_mask).long().to(gpu)
    labels = torch.from_numpy(ds.labels).long().to(gpu)
    m = build_model(cfg, task="masked-lm", seed=0).to(gpu)
    store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, fp8=True)
    hip.set_fp8(True)
    prev = hip._FP8_WGRAD
    out = {}
    try:
        for step, w8 in enumerate((False, False, False, True)):
            hip._FP8_WGRAD = w8
            n0 = hip.WGRAD8_CALLS[0]
            m.train()
            m.rng.new_step(0)
            store.zero_grad()
            loss, _ = m(ids, attention_mask=am, labels=labels)
            loss.backward()
            torch.cuda.synchronize()
            out[w8] = store.grad.float().clone()
            if step < 2:
                store.refresh_fp8()
            if w8:
                assert hip.WGRAD8_CALLS[0] - n0 == 8
    finally:
        hip._FP8_WGRAD = prev
        hip.set_fp8(False)
    g0, g1 = out[False], out[True]
    assert torch.isfinite(g1).all()
    cos = torch.nn.functional.cosine_similarity(g0, g1, dim=0)
    assert cos > 0.995, float(cos)
    rel = float((g1 - g0).norm() / g0.norm())
    assert rel < 0.1, rel


@pytest.mark.parametrize("B_,S,heads,K,fa", [(4, 512, 16, 1024, 0), (3, 384, 12, 768, 1)])
def test_gemm8_row_dot_epilogue(gpu, B_, S, heads, K, fa):
    """fp8 out-projection dgrad with the attention backward's delta rows (E2_STORE_RDOT on gemm8pk): dx bit-identical
    to the plain store epilogue, the rows bit-identical to the streaming attention's own delta pass, and the fp8
    attention backward fed them (delta_ready) bit-identical to the one that computes them."""
    hip = _hip()
    C = hip._C
    torch.manual_seed(3 + K)
    H = heads * 64
    T = B_ * S
    dy = torch.randn(T, K, device=gpu).bfloat16()
    wt = (torch.randn(H, K, device=gpu) * 0.05).bfloat16()  # Wᵀ [N][K]
    qdy, sdy = hip.quant_fp8(dy, fa)
    qw, sw = hip.quant_fp8(wt, 0)
    qkv = torch.randn(T, 3 * H, device=gpu).bfloat16()
    o = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    lse = torch.empty(B_ * heads * S, device=gpu)
    C.attn_fwd(qkv, None, o, lse, B_, S, heads, 0.1, 7)
    dx0 = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    C.gemm8(qdy, fa, sdy, qw, 0, sw, dx0, 0)
    dx1 = torch.empty_like(dx0)
    rd = torch.full((B_ * heads * S,), float("nan"), device=gpu)
    C.gemm8(qdy, fa, sdy, qw, 0, sw, dx1, 10, None, o, rd=rd, rd_seq=S)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    outs = []
    for ready in (False, True):
        ws = rd.clone() if ready else torch.empty_like(rd)
        dqkv = torch.empty_like(qkv)
        gst = torch.tensor([3.0, 0.0], device=gpu)
        gq, gs = torch.empty(T, 3 * H, dtype=torch.uint8, device=gpu), torch.empty(1, device=gpu)
        C.attn_bwd_q8(qkv, None, o, dx0, lse, dqkv, ws, B_, S, heads, 0.1, 7, None, gq, gst[0:1], gs, gst[1:2], 0,
                      None, ready)
        torch.cuda.synchronize()
        outs.append((ws, dqkv, gq))
    assert torch.equal(outs[0][0], rd)
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])


def test_fp8_weight_copies_requantised_per_slice_match_one_pass(gpu, monkeypatch):
    """Overlapped optimizer slices re-quantise their own fp8 weights (W8, W8ᵀ, scale) right after each update
    (FlatParamStore.fp8_subsets / refresh_fp8_subset): after every step the copies equal one refresh_fp8 pass over all
    weights from the same bf16 copies, bit for bit."""
    from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata
    from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config
    from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam
    from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore
    from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer

    hip = _hip()
    monkeypatch.setenv("HSD_OPT_BUCKET_MB", "4")
    cfg = resolve_config("roberta-large").replace(num_hidden_layers=2)
    ds = hdata.synthetic_mlm(8, 256, cfg.vocab_size, seed=5)
    batch = {"input_ids": torch.from_numpy(ds.input_ids).long().to(gpu),
             "attention_mask": torch.from_numpy(ds.attention_mask).long().to(gpu),
             "labels": torch.from_numpy(ds.labels).long().to(gpu)}
    m = build_model(cfg, task="masked-lm", seed=0).to(gpu)
    hip.set_fp8(True)
    try:
        store = FlatParamStore(m, gpu, compute_dtype=torch.bfloat16, fp8=True)
        opt = FusedAdam(store, lr=1e-4)
        tr = Trainer(m, store, opt, None, gpu)
        assert opt._f8sub is not None and sum(x is not None for x in opt._f8sub) >= 2
        for _ in range(3):
            tr.train_step([batch])
            torch.cuda.synchronize()
            q, qt, si = store.fp8_w.clone(), store.fp8_wt.clone(), store.fp8_sinv.clone()
            store.refresh_fp8()
            torch.cuda.synchronize()
            assert torch.equal(q, store.fp8_w) and torch.equal(qt, store.fp8_wt) and torch.equal(si, store.fp8_sinv)
            assert int(torch.count_nonzero(store.fp8_amax)) == 0
    finally:
        hip.set_fp8(False)
