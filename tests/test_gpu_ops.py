"""HIP kernel numerics vs the plain-PyTorch fp32 reference of the same op (SURVEY.md §4 'kernel / GPU').

Dropout masks are bit-identical between the kernels and ops/reference.py (shared hash), so every
test also runs with dropout on.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from huggingface_sagemaker_tensorflow_distributed_amd.ops import reference as ref  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.ops.rng import keep_mask  # noqa: E402


def _hip():
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip

    return hip


def _close(a, b, atol, rtol, what=""):
    """At most 0.1 % of the elements beyond tolerance (bf16 rounding flips), and NONE beyond 4x the tolerance."""
    a = a.float()
    b = b.float()
    err = (a - b).abs()
    # atol is relative to the tensor's scale (bf16 outputs of long reductions), rtol per element
    tol = atol * b.abs().max().clamp_min(1e-6) + rtol * b.abs()
    bad = (err > tol).float().mean().item()
    worst = (err / tol).max().item()
    assert bad <= 1e-3, f"{what}: {bad*100:.3f}% elements out of tol, max err {err.max().item():.4g}"
    assert worst <= 4.0, f"{what}: an element is {worst:.2f}x beyond tolerance (max err {err.max().item():.4g})"


def test_extension_loaded(gpu):
    hip = _hip()
    assert hip._C.__file__.endswith(".so")


def test_dropout_mask_matches_reference(gpu):
    hip = _hip()
    x = torch.ones(4096 * 3, device=gpu, dtype=torch.bfloat16)
    seed = 0xDEADBEEF12345678
    y = hip.dropout(x, 0.1, seed)
    m = keep_mask(seed, x.shape, 0.1, device=gpu)
    assert torch.equal(y.float() != 0, m)
    frac = m.float().mean().item()
    assert abs(frac - 0.9) < 0.02


@pytest.mark.parametrize("H", [64, 768, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_dense_residual_ln(gpu, H, p):
    hip = _hip()
    torch.manual_seed(0)
    T, K = 512, 256
    x = torch.randn(T, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(H, K, device=gpu) * 0.05).bfloat16().requires_grad_()
    b = (torch.randn(H, device=gpu) * 0.1).bfloat16().requires_grad_()
    res = torch.randn(T, H, device=gpu, dtype=torch.bfloat16)
    g = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    be = (0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    xr = x.clone().requires_grad_()
    rr = res.clone().requires_grad_()
    out = hip.dense_residual_ln(xr, w, b, rr, g, be, 1e-12, p, 1234)
    # reference in fp32
    x32, w32, b32, r32, g32, be32 = [t.detach().float().requires_grad_() for t in (x, w, b, res, g, be)]
    ref_out = ref.layer_norm(ref.linear_dropout_residual(x32, w32, b32, r32, p, 1234, p > 0), g32, be32, 1e-12)
    _close(out, ref_out, 3e-2, 2e-2, "fwd")
    dout = torch.randn_like(out)
    out.backward(dout)
    ref_out.backward(dout.float())
    _close(xr.grad, x32.grad, 5e-2, 5e-2, "dx")
    _close(rr.grad, r32.grad, 5e-2, 5e-2, "dres")
    _close(w.grad, w32.grad, 5e-2, 5e-2, "dw")
    _close(b.grad, b32.grad, 1e-1, 2e-2, "db")
    _close(g.grad, g32.grad, 1e-1, 2e-2, "dgamma")
    _close(be.grad, be32.grad, 1e-1, 2e-2, "dbeta")


def test_linear_gelu(gpu):
    hip = _hip()
    torch.manual_seed(1)
    T, K, N = 1024, 256, 512
    x = torch.randn(T, K, device=gpu, dtype=torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=gpu) * 0.05).bfloat16().requires_grad_()
    b = (torch.randn(N, device=gpu) * 0.1).bfloat16().requires_grad_()
    y = hip.linear_gelu(x, w, b)
    x32, w32, b32 = [t.detach().float().requires_grad_() for t in (x, w, b)]
    yr = ref.linear_gelu(x32, w32, b32)
    _close(y, yr, 2e-2, 2e-2, "fwd")
    d = torch.randn_like(y)
    y.backward(d)
    yr.backward(d.float())
    _close(x.grad, x32.grad, 5e-2, 5e-2, "dx")
    _close(w.grad, w32.grad, 1e-1, 5e-2, "dw")
    _close(b.grad, b32.grad, 2e-1, 2e-2, "db")


@pytest.mark.parametrize("H", [64, 256, 768, 1024])
def test_layer_norm_plain(gpu, H):
    """LN without residual / dropout (the encoder tails' LN, 16-B multi-row forward kernel) vs fp32 torch."""
    hip = _hip()
    torch.manual_seed(5)
    T = 4099  # not a multiple of the rows-per-wave / waves-per-block tiling
    x = torch.randn(T, H, device=gpu).bfloat16().requires_grad_()
    g = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    out = hip.layer_norm(x, g, b, 1e-12)
    x32, g32, b32 = [t.detach().float().requires_grad_() for t in (x, g, b)]
    r = torch.nn.functional.layer_norm(x32, (H,), g32, b32, 1e-12)
    _close(out, r, 3e-2, 2e-2, "fwd")
    d = torch.randn_like(out)
    out.backward(d)
    r.backward(d.float())
    _close(x.grad, x32.grad, 5e-2, 5e-2, "dx")
    _close(g.grad, g32.grad, 2e-1, 2e-2, "dgamma")
    _close(b.grad, b32.grad, 2e-1, 2e-2, "dbeta")


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("type_vocab", [2, 0])
@pytest.mark.parametrize("arange", [True, False])
def test_embed_ln(gpu, p, type_vocab, arange):
    hip = _hip()
    torch.manual_seed(2)
    B, S, H, V = 8, 64, 768, 1000
    ids = torch.randint(0, V, (B, S), device=gpu)
    # RoBERTa-style position ids (padding_idx + 1 + arange, per-token gradient atomics) when not arange
    pos = torch.arange(S, device=gpu).unsqueeze(0).expand(B, S) + (0 if arange else 2)
    tt = torch.randint(0, 2, (B, S), device=gpu) if type_vocab else None
    word = (torch.randn(V, H, device=gpu) * 0.02).bfloat16().requires_grad_()
    pw = (torch.randn(S + 2, H, device=gpu) * 0.02).bfloat16().requires_grad_()
    tw = (torch.randn(2, H, device=gpu) * 0.02).bfloat16().requires_grad_() if type_vocab else None
    g = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    be = (0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    out = hip.embed_ln(ids, pos, tt, word, pw, tw, g, be, 1e-12, p, 99, arange)
    f = lambda t: t.detach().float().requires_grad_() if t is not None else None  # noqa: E731
    word32, pw32, tw32, g32, be32 = f(word), f(pw), f(tw), f(g), f(be)
    r = ref.embed_ln(ids, pos, tt, word32, pw32, tw32, g32, be32, 1e-12, 0.0, 0, False)
    if p > 0:
        # kernel applies dropout to the bf16-rounded LN output
        r = r.bfloat16().float() * keep_mask(99, r.shape, p, device=gpu).float() / (1 - p)
    _close(out, r, 3e-2, 2e-2, "fwd")
    d = torch.randn_like(out)
    out.backward(d)
    r.backward(d.float())
    _close(word.grad, word32.grad, 1e-2, 5e-2, "dword")
    _close(pw.grad, pw32.grad, 1e-1, 5e-2, "dpos")
    if type_vocab:
        _close(tw.grad, tw32.grad, 5e-1, 5e-2, "dtype")
    _close(g.grad, g32.grad, 2e-1, 5e-2, "dgamma")
    _close(be.grad, be32.grad, 2e-1, 5e-2, "dbeta")


@pytest.mark.parametrize("S", [32, 128, 256, 384, 512])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("masked", [False, True])
def test_attention(gpu, S, p, masked):
    hip = _hip()
    torch.manual_seed(3)
    B, heads = 4, 4
    H = heads * 64
    qkv = torch.randn(B * S, 3 * H, device=gpu, dtype=torch.bfloat16).requires_grad_()
    mb = None
    if masked:
        lens = torch.randint(S // 4, S + 1, (B,), device=gpu)
        am = (torch.arange(S, device=gpu)[None, :] < lens[:, None]).long()
        mb = ref.key_mask_bias(am)
    out = hip.attention(qkv, mb, B, S, heads, p, 777)
    q32 = qkv.detach().float().requires_grad_()
    r = ref.attention(q32, mb, B, S, heads, p, 777, p > 0)
    _close(out, r, 2e-2, 2e-2, "fwd")
    d = torch.randn_like(out)
    out.backward(d)
    r.backward(d.float())
    g, gr = qkv.grad.float(), q32.grad
    for i, name in enumerate("qkv"):
        _close(g[:, i * H:(i + 1) * H], gr[:, i * H:(i + 1) * H], 3e-2, 3e-2, f"d{name}")


def test_adam_kernel_matches_reference(gpu):
    hip = _hip()
    torch.manual_seed(4)
    n = 4096
    p = torch.randn(n, device=gpu)
    m = torch.randn(n, device=gpu).abs() * 0.1
    v = torch.randn(n, device=gpu).abs() * 0.1
    g = torch.randn(n, device=gpu)
    out = torch.empty(n, device=gpu, dtype=torch.bfloat16)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    step, eps, b1, b2, gs = 1e-3, 1e-7, 0.9, 0.999, 0.5
    hip.adam_step(p, m, v, g, out, None, step, eps, b1, b2, gs, 0.0)
    gg = g * gs
    mr = b1 * mr + (1 - b1) * gg
    vr = b2 * vr + (1 - b2) * gg * gg
    pr = pr - step * mr / (vr.sqrt() + eps)
    torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out.float(), pr.bfloat16().float())


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_adam_kernel_zero_grad_clears_what_it_read(gpu, gdt):
    """zero_grad=True: the same weights / moments / bf16 copy bit for bit, and the gradient slice left at zero (the
    slice only: the elements around it untouched)."""
    hip = _hip()
    torch.manual_seed(6)
    n = 64 * 1024
    base = [torch.randn(n, device=gpu), torch.randn(n, device=gpu).abs() * 0.1, torch.randn(n, device=gpu).abs() * 0.1]
    gfull = torch.randn(n + 2048, device=gpu).to(gdt)
    res = {}
    for zg in (False, True):
        p, m, v = (t.clone() for t in base)
        g = gfull.clone()
        out = torch.empty(n, device=gpu, dtype=torch.bfloat16)
        hip.adam_step(p, m, v, g[1024:1024 + n], out, None, 1e-3, 1e-7, 0.9, 0.999, 0.5, 0.0, zero_grad=zg)
        torch.cuda.synchronize()
        res[zg] = (p, m, v, out, g)
    for a, b in zip(res[False][:4], res[True][:4]):
        assert torch.equal(a, b)
    g0, g1 = res[False][4], res[True][4]
    assert torch.equal(g0, gfull)
    assert bool((g1[1024:1024 + n] == 0).all())
    assert torch.equal(g1[:1024], gfull[:1024]) and torch.equal(g1[1024 + n:], gfull[1024 + n:])


@pytest.mark.parametrize("S,H,heads", [(128, 256, 4), (256, 256, 4), (128, 1024, 16), (512, 1024, 16)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_blocks_vs_reference(gpu, p, S, H, heads):
    """attn_block / ffn_block (GEMM epilogues + fused backward) vs composed fp32 reference ops.
    S = 128 runs attention128.hip, S = 256 / 512 the streaming kernels of attentionS.hip (incl. the fused
    qkv bias gradient of both); H = 1024 with 16 heads is bert-large's width."""
    hip = _hip()
    torch.manual_seed(5)
    B, I = (4 if H == 256 else 2), 4 * H
    T = B * S
    mk = lambda *s, sc=0.05: (torch.randn(*s, device=gpu) * sc).bfloat16().requires_grad_()  # noqa: E731
    h = torch.randn(T, H, device=gpu).bfloat16().requires_grad_()
    qw, qb, ow, ob = mk(3 * H, H), mk(3 * H), mk(H, H), mk(H)
    lw, lb = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_(), mk(H)
    w1, b1, w2, b2 = mk(I, H), mk(I), mk(H, I), mk(H)
    l2w, l2b = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_(), mk(H)
    am = torch.ones(B, S, dtype=torch.long, device=gpu)
    am[B // 2, 100:] = 0
    mb = ref.key_mask_bias(am)
    params = [h, qw, qb, ow, ob, lw, lb, w1, b1, w2, b2, l2w, l2b]

    def run(hip_path):
        for t in params:
            t.grad = None
        if hip_path:
            h1 = hip.attn_block(h, qw, qb, ow, ob, lw, lb, 1e-12, mb, B, S, heads, p, 11, p, 12)
            out = hip.ffn_block(h1, w1, b1, w2, b2, l2w, l2b, 1e-12, p, 13)
        else:
            f = [t.detach().float().requires_grad_() for t in params]
            qkv = ref.linear(f[0], f[1], f[2])
            ctx_ = ref.attention(qkv, mb, B, S, heads, p, 11, p > 0)
            h1 = ref.layer_norm(ref.linear_dropout_residual(ctx_, f[3], f[4], f[0], p, 12, p > 0), f[5], f[6], 1e-12)
            a = ref.linear_gelu(h1, f[7], f[8])
            out = ref.layer_norm(ref.linear_dropout_residual(a, f[9], f[10], h1, p, 13, p > 0), f[11], f[12], 1e-12)
            params_f = f
        g = torch.randn(out.shape, device=gpu, generator=torch.Generator(device=gpu).manual_seed(9))
        out.backward(g.to(out.dtype))
        grads = [t.grad.float() for t in (params if hip_path else params_f)]
        return out.float(), grads

    o1, g1 = run(True)
    o2, g2 = run(False)
    _close(o1, o2, 3e-2, 3e-2, "out")
    names = ["h", "qw", "qb", "ow", "ob", "lw", "lb", "w1", "b1", "w2", "b2", "l2w", "l2b"]
    for n, a, b in zip(names, g1, g2):
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 4e-2, f"{n}: rel err {rel:.3g}"


@pytest.mark.parametrize("S", [128, 256, 512])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_fast_paths_match_generic_kernel(gpu, p, S, monkeypatch):
    """The S == 128 one-workgroup-per-head kernels (attention128.hip) and the S > 128 streaming kernels
    (attentionS.hip) vs the tiled generic kernels (same dropout masks, so tight tolerances)."""
    hip = _hip()
    torch.manual_seed(7)
    B, heads = 3, 12
    H = heads * 64
    qkv = torch.randn(B * S, 3 * H, device=gpu, dtype=torch.bfloat16)
    am = torch.ones(B, S, dtype=torch.long, device=gpu)
    am[1, 77:] = 0
    mb = ref.key_mask_bias(am)
    d = torch.randn(B * S, H, device=gpu, dtype=torch.bfloat16)
    outs = []
    try:
        for generic in (False, True):
            hip._C.attn_set_force_generic(generic)
            x = qkv.clone().requires_grad_()
            o = hip.attention(x, mb, B, S, heads, p, 4242)
            o.backward(d)
            outs.append((o.float(), x.grad.float()))
    finally:
        hip._C.attn_set_force_generic(False)
    _close(outs[0][0], outs[1][0], 1e-2, 1e-2, "fwd")
    _close(outs[0][1], outs[1][1], 2e-2, 2e-2, "bwd")


@pytest.mark.parametrize("S", [256, 512])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_keep_mask_matches_rehash(gpu, masked, S):
    """The forward's dropout keep bits (ballot words, _keep_mask) read by the backward == the backward that re-hashes
    every (query, key) pair (the streaming dK/dV and dQ passes, attentionS.hip): identical output and dqkv, bit for bit
    (the atomically summed bias gradient to fp32 rounding)."""
    hip = _hip()
    C_ = hip._C
    torch.manual_seed(11 + S)
    B, heads, p = 3, 12, 0.1
    H = heads * 64
    qkv = torch.randn(B * S, 3 * H, device=gpu, dtype=torch.bfloat16)
    mb = None
    if masked:
        am = torch.ones(B, S, dtype=torch.long, device=gpu)
        am[2, 50:] = 0
        am[0, S - 70:] = 0
        mb = ref.key_mask_bias(am).float().contiguous()
    dout = torch.randn(B * S, H, device=gpu, dtype=torch.bfloat16)
    res = []
    for use_km in (False, True):
        out = torch.empty(B * S, H, device=gpu, dtype=torch.bfloat16)
        lse = torch.empty(B * heads * S, device=gpu)
        km = hip._keep_mask(B, S, heads, p, gpu) if use_km else None
        assert (km is not None) == use_km
        C_.attn_fwd(qkv, mb, out, lse, B, S, heads, p, 99, km)
        dqkv = torch.empty_like(qkv)
        db = torch.zeros(3 * H, device=gpu)
        ws = hip._attn_ws(B, S, heads, gpu)
        C_.attn_bwd(qkv, mb, out, dout, lse, dqkv, ws, B, S, heads, p, 99, db, km)
        torch.cuda.synchronize()
        res.append((out, dqkv, db, km))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    # the bias gradient is summed by fp32 atomics across workgroups: equal up to the order of those additions
    torch.testing.assert_close(res[1][2], res[0][2], rtol=1e-5, atol=1e-5 * float(res[0][2].abs().max()))
    # ~90 % of the bits set (p = 0.1)
    km = res[1][3]
    ones = sum(bin(int(w) & 0xFFFFFFFF).count("1") for w in km[:4096].cpu().tolist())
    assert 0.88 < ones / (4096 * 32) < 0.92


@pytest.mark.parametrize("R,V,dtype", [(64, 2, torch.float32), (300, 2, torch.bfloat16), (97, 50265, torch.bfloat16),
                                       (33, 1003, torch.float32)])
def test_fused_cross_entropy(gpu, R, V, dtype):
    """xent.hip: loss, gradient and argmax-correct count vs torch (ignore_index -100)."""
    hip = _hip()
    torch.manual_seed(8)
    logits = (torch.randn(R, V, device=gpu) * 3).to(dtype).requires_grad_()
    labels = torch.randint(0, V, (R,), device=gpu)
    labels[::5] = -100
    loss, correct = hip.cross_entropy(logits, labels)
    loss.backward()
    l32 = logits.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(l32, labels, ignore_index=-100)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    _close(logits.grad, l32.grad, 2e-2 if dtype == torch.bfloat16 else 1e-5, 1e-3, "dlogits")
    keep = labels.ne(-100)
    assert int(correct.item()) == int((l32.argmax(-1) == labels)[keep].sum().item())


@pytest.mark.parametrize("model", ["bert", "roberta", "distilbert"])
@pytest.mark.parametrize("B,C,H", [(8, 2, 1024), (256, 2, 768), (64, 3, 768)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_cls_head_vs_reference(gpu, model, B, C, H, p):
    """ops.cls_head on GPU (dense on gemm2 + cls_head.hip fused act / dropout / classifier / CE / accuracy, fused
    backward with dW2 / db2 atomics, dgrad written into the [CLS] rows of dh) vs the fp32 reference head + CE."""
    from huggingface_sagemaker_tensorflow_distributed_amd import ops

    torch.manual_seed(17)
    S = 16
    mk = lambda *s, sc=0.05: (torch.randn(*s, device=gpu) * sc).bfloat16().requires_grad_()  # noqa: E731
    h = torch.randn(B, S, H, device=gpu).bfloat16().requires_grad_()
    w1, b1, w2, b2 = mk(H, H), mk(H, sc=0.5), mk(C, H, sc=0.5), mk(C, sc=0.5)
    labels = torch.randint(0, C, (B,), device=gpu)
    labels[1] = -100  # an ignored row (eval-shard padding)
    act = "relu" if model == "distilbert" else "tanh"
    p_in = p if model == "roberta" else 0.0
    params = [h, w1, b1, w2, b2]
    loss, logits = ops.cls_head(h, w1, b1, w2, b2, labels, act, p_in, 21, p, 22)
    assert getattr(loss, "_hsd_stats", None) is not None, "the fused HIP head did not run"
    loss.backward()
    g_hip = [t.grad.float() for t in params]
    f = [t.detach().float().requires_grad_() for t in params]
    lg_ref = ref.cls_head(f[0][:, 0], f[1], f[2], f[3], f[4], act, p_in, 21, p, 22, True)
    loss_ref = torch.nn.functional.cross_entropy(lg_ref, labels, ignore_index=-100)
    loss_ref.backward()
    assert abs(loss.item() - loss_ref.item()) < 2e-2 * max(1.0, abs(loss_ref.item())), (loss.item(), loss_ref.item())
    _close(logits, lg_ref, 3e-2, 3e-2, "logits")
    valid = labels.ne(-100)
    hits = (lg_ref.argmax(-1) == labels)[valid].sum().item()
    assert abs(loss._hsd_stats[1].item() - hits) <= 1 and loss._hsd_stats[2].item() == valid.sum().item()
    for n, a, b in zip(["h", "w1", "b1", "w2", "b2"], g_hip, [t.grad for t in f]):
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 4e-2, f"{n}: rel err {rel:.3g}"
    assert torch.count_nonzero(g_hip[0][:, 1:]) == 0  # only the first-token rows receive gradient


@pytest.mark.parametrize("H", [256, 1024])
def test_mlm_head_vs_reference(gpu, H):
    """The masked-LM head at RoBERTa's vocabulary (V = 50265, padded to 50432 inside the model): every GEMM on gemm2
    (no library GEMM), CE over the real vocabulary only, vs the fp32 reference on the unpadded table."""
    from huggingface_sagemaker_tensorflow_distributed_amd import ops

    torch.manual_seed(23)
    V, Vp, T = 50265, 50432, 512
    mk = lambda *s, sc=0.05: (torch.randn(*s, device=gpu) * sc).bfloat16()  # noqa: E731
    h = torch.randn(T, H, device=gpu).bfloat16().requires_grad_()
    w1, b1 = mk(H, H).requires_grad_(), mk(H).requires_grad_()
    lw = (1 + 0.1 * torch.randn(H, device=gpu)).bfloat16().requires_grad_()
    lb = mk(H).requires_grad_()
    wemb = mk(Vp, H)
    wemb[V:] = 0
    wemb.requires_grad_()
    bias = mk(Vp)
    bias[V:] = 0
    bias.requires_grad_()
    labels = torch.full((T,), -100, device=gpu, dtype=torch.long)
    m = torch.rand(T, device=gpu) < 0.15
    labels[m] = torch.randint(0, V, (int(m.sum()),), device=gpu)
    params = [h, w1, b1, lw, lb, wemb, bias]
    loss, logits = ops.mlm_head(h, labels, w1, b1, lw, lb, 1e-5, wemb, bias, V)
    assert getattr(loss, "_hsd_correct", None) is not None, "the fused HIP head did not run"
    assert logits.shape == (int(m.sum()), V)
    loss.backward()
    g_hip = [t.grad.float() for t in params]
    f = [t.detach().float().requires_grad_() for t in params]
    loss_ref, lg_ref = ref.mlm_head(f[0], labels, f[1], f[2], f[3], f[4], 1e-5, f[5], f[6], V)
    loss_ref.backward()
    assert abs(loss.item() - loss_ref.item()) < 1e-2 * abs(loss_ref.item()), (loss.item(), loss_ref.item())
    _close(logits, lg_ref, 3e-2, 3e-2, "logits")
    for n, a, b in zip(["h", "w1", "b1", "ln_w", "ln_b", "wemb", "bias"], g_hip, [t.grad for t in f]):
        rel = (a - b).norm() / (b.norm() + 1e-6)
        assert rel < 5e-2, f"{n}: rel err {rel:.3g}"
    assert torch.count_nonzero(g_hip[5][V:]) == 0 and torch.count_nonzero(g_hip[6][V:]) == 0  # padding stays 0
