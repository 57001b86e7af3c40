"""MFMA GEMM (csrc/kernels/gemm.hip) vs a plain fp32 PyTorch reference: all layouts and epilogues."""
import pytest
import torch

pytestmark = pytest.mark.gpu

EPI_STORE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_DROP_RES, EPI_RES, EPI_DGELU, EPI_F32_ATOMIC = range(7)


def _C():
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip

    return hip._C


def _mk(shape, dev, scale=1.0):
    return (torch.randn(shape, device=dev) * scale).bfloat16()


def _ref(A, B, la, lb):
    a = A.float() if la == 0 else A.float().t()
    b = B.float() if lb == 1 else B.float().t()
    return a @ b  # [M, N]


def _check(out, ref, mag=None, acc=None, fp32=False):
    """Per-element bound (a max-relative 2 % bound let a wrong edge tile at 1 % of the max pass):

        |out - ref| <= rel * mag + 2^-16 * acc + 1e-30

    * rel = 2^-7 for bf16 outputs: one bf16 ulp of each rounded intermediate (the kernel and the reference may round
      values that differ in the last fp32 bits to neighbouring bf16 values); 2^-20 for fp32 outputs.
    * mag: elementwise magnitude of the rounded intermediates (default |ref|; epilogues pass |pre-activation| etc.).
    * acc: elementwise sum of |products| (|A| @ |B|), which bounds fp32 accumulation-order differences from torch's
      GEMM (~sqrt(K) * 2^-24 * acc typical, 2^-16 * acc is 2^8 above that)."""
    out = out.float()
    mag = ref.abs() if mag is None else mag
    bound = (2.0 ** -20 if fp32 else 2.0 ** -7) * mag + 1e-30
    if acc is not None:
        bound = bound + 2.0 ** -16 * acc
    err = (out - ref).abs()
    bad = err > bound
    if bad.any():
        i = int(bad.flatten().nonzero()[0])
        raise AssertionError(f"{int(bad.sum())} of {bad.numel()} elements out of bound; first at flat index {i}: "
                             f"out {out.flatten()[i].item():.6g} ref {ref.flatten()[i].item():.6g} "
                             f"bound {bound.flatten()[i].item():.3g} (max err {err.max().item():.4g})")


def _absmm(A, B, la, lb):
    """|A| @ |B| in the layout of _ref: the accumulation magnitude of every output element."""
    return _ref(A.abs(), B.abs(), la, lb)


SHAPES = [(256, 256, 128), (200, 136, 72), (1024, 768, 768), (512, 2304, 64), (96, 64, 3072)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1)])
def test_gemm_store(gpu, M, N, K, la, lb):
    torch.manual_seed(0)
    A = _mk((M, K) if la == 0 else (K, M), gpu)
    B = _mk((N, K) if lb == 0 else (K, N), gpu)
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    _C().gemm(A, B, C, la, lb, EPI_STORE, None, None, None, 0.0, 0, 1)
    _check(C, _ref(A, B, la, lb), acc=_absmm(A, B, la, lb))


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("la,lb", [(1, 1), (0, 0), (0, 1)])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_f32_atomic_accumulates(gpu, M, N, K, la, lb, splits):
    torch.manual_seed(1)
    A = _mk((M, K) if la == 0 else (K, M), gpu)
    B = _mk((N, K) if lb == 0 else (K, N), gpu)
    C0 = torch.randn(M, N, device=gpu)
    C = C0.clone()
    _C().gemm(A, B, C, la, lb, EPI_F32_ATOMIC, None, None, None, 0.0, 0, splits)
    _check(C, C0 + _ref(A, B, la, lb), acc=_absmm(A, B, la, lb) + C0.abs(), fp32=True)


def test_gemm_bias_epilogues(gpu):
    torch.manual_seed(2)
    M, N, K = 384, 512, 256
    A, B = _mk((M, K), gpu), _mk((N, K), gpu, 0.1)
    bias = _mk((N,), gpu)
    ref = _ref(A, B, 0, 0) + bias.float()
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    acc = _absmm(A, B, 0, 0)
    _C().gemm(A, B, C, 0, 0, EPI_BIAS, bias, None, None, 0.0, 0, 1)
    _check(C, ref, acc=acc)
    C2 = torch.empty_like(C)
    _C().gemm(A, B, C, 0, 0, EPI_BIAS_GELU, bias, None, C2, 0.0, 0, 1)
    _check(C, ref, acc=acc)
    g = torch.nn.functional.gelu(ref)
    _check(C2, g, mag=2 * ref.abs() + g.abs(), acc=2 * acc)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_bias_dropout_residual(gpu, p):
    from huggingface_sagemaker_tensorflow_distributed_amd.ops.reference import dropout

    torch.manual_seed(3)
    M, N, K = 256, 768, 512
    A, B = _mk((M, K), gpu), _mk((N, K), gpu, 0.05)
    bias, res = _mk((N,), gpu), _mk((M, N), gpu)
    y = (_ref(A, B, 0, 0) + bias.float()).bfloat16()
    ref = dropout(y.float(), p, 4242, True) + res.float()  # one rounding, as the kernels
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    _C().gemm(A, B, C, 0, 0, EPI_BIAS_DROP_RES, bias, res, None, p, 4242, 1)
    _check(C, ref, mag=2 * y.float().abs() + res.float().abs() + ref.abs(), acc=2 * _absmm(A, B, 0, 0))


@pytest.mark.parametrize("M", [96, 512])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_dropout_residual_site_same_bits_on_every_gemm_path(gpu, M, p):
    """the dropout + residual epilogue rounds once, bf16(fma(y, keep·scale, residual)), on every kernel that
    serves the site -- gemm2 (the NT fast path), gemm.hip's LDS-DMA kernel (M >= 128) and its register-staged kernel
    (M < 128), the fallbacks `gemm_fwd` takes when `_nt_ok` fails. Small-integer operands make the fp32 accumulation
    exact in any order, so y = bf16(acc + b) is the same on every path and the outputs must match bit for bit."""
    torch.manual_seed(5)
    N, K = 768, 128
    A = torch.randint(-1, 2, (M, K), device=gpu).bfloat16()
    B = torch.randint(-1, 2, (N, K), device=gpu).bfloat16()
    bias = torch.randint(-2, 3, (N,), device=gpu).bfloat16()
    res = _mk((M, N), gpu)
    outs = []
    for kernel in ("gemm", "gemm2"):
        C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        if kernel == "gemm":
            _C().gemm(A, B, C, 0, 0, EPI_BIAS_DROP_RES, bias, res, None, p, 777, 1)
        else:
            _C().gemm2(A, B, C, 0, 0, EPI_BIAS_DROP_RES, bias, res, None, p, 777, 1, None, None)
        outs.append(C)
    assert torch.equal(outs[0], outs[1]), int((outs[0] != outs[1]).sum())
    from huggingface_sagemaker_tensorflow_distributed_amd.ops.reference import keep_mask

    y = (A.float() @ B.float().t() + bias.float()).bfloat16().float()
    k = keep_mask(777, (M, N), p, device=gpu).float() * (1.0 / (1.0 - p)) if p > 0 else torch.ones_like(y)
    ref = torch.addcmul(res.float(), y, k).bfloat16()
    # fp32 fma vs torch's product-then-sum: the same bf16 value except on a rare fp32 tie
    assert float((outs[0].float() != ref.float()).float().mean()) < 1e-3


def test_gemm_dgrad_epilogues(gpu):
    torch.manual_seed(4)
    M, N, K = 512, 768, 1024  # dX[M,N] = dY[M,K] . W[K,N]
    A, B = _mk((M, K), gpu), _mk((K, N), gpu, 0.05)
    aux = _mk((M, N), gpu)
    ref = _ref(A, B, 0, 1)
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    acc = _absmm(A, B, 0, 1)
    _C().gemm(A, B, C, 0, 1, EPI_RES, None, aux, None, 0.0, 0, 1)
    _check(C, ref + aux.float(), mag=ref.abs() + aux.float().abs() + (ref + aux.float()).abs(), acc=acc)
    _C().gemm(A, B, C, 0, 1, EPI_DGELU, None, aux, None, 0.0, 0, 1)
    x = aux.float().requires_grad_()
    torch.nn.functional.gelu(x).backward(torch.ones_like(x))
    r = ref.bfloat16().float() * x.grad
    _check(C, r, mag=ref.abs() * x.grad.abs() * 2 + r.abs(), acc=acc * 2)


# ---------------------------------------------------------------- gemm2 (8-phase 256-row tiles)
G2_SHAPES = [(256, 768, 768), (300, 768, 128), (1000, 960, 192), (512, 2304, 256), (768, 3072, 512)]


def _gelu_grad(x):
    import math

    return 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)


@pytest.mark.parametrize("M,N,K", G2_SHAPES)
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5])
def test_gemm2_nt_epilogues(gpu, M, N, K, epi):
    from huggingface_sagemaker_tensorflow_distributed_amd.ops import reference as ref

    torch.manual_seed(11 + epi)
    C_ = _C()
    A, B = _mk((M, K), gpu), _mk((N, K), gpu, 0.1)
    bias, aux = _mk((N,), gpu), _mk((M, N), gpu)
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    C2 = torch.empty_like(C)
    p = 0.1 if epi == 3 else 0.0
    C_.gemm2(A, B, C, 0, 0, epi, bias if epi in (1, 2, 3) else None, aux if epi in (3, 4, 5) else None,
             C2 if epi == 2 else None, p, 99, 1, None, None)
    acc = A.float() @ B.float().t()
    am = _absmm(A, B, 0, 0)
    if epi in (1, 2, 3):
        acc = acc + bias.float()
    if epi == 2:
        _check(C, acc, acc=am)
        g = torch.nn.functional.gelu(C.float())
        _check(C2, g, mag=2 * C.float().abs() + g.abs())
        return
    mag = acc.abs()
    if epi == 3:
        y = acc.bfloat16().float()
        keep = ref.dropout(torch.ones(M, N, device=gpu), p, 99, True)
        acc = y * keep + aux.float()  # one rounding (gemm_common.h E2_BIAS_DROP_RES)
        mag = 2 * (y * keep).abs() + aux.float().abs() + acc.abs()
    elif epi == 4:
        acc = acc.bfloat16().float() + aux.float()
        mag = mag + aux.float().abs() + acc.abs()
    elif epi == 5:
        gg = _gelu_grad(aux.float())
        acc = acc.bfloat16().float() * gg
        mag = 2 * mag * gg.abs() + acc.abs()
    _check(C, acc, mag=mag, acc=2 * am)


@pytest.mark.parametrize("M,N,K", [(768, 768, 256), (2304, 768, 512), (256, 1024, 4096)])
@pytest.mark.parametrize("epi", [6, 7])
def test_gemm2_tt_wgrad(gpu, M, N, K, epi):
    torch.manual_seed(12)
    C_ = _C()
    A, B = _mk((K, M), gpu), _mk((K, N), gpu)
    C0 = torch.randn(M, N, device=gpu)
    C = C0.clone()
    sp = C_.gemm2_splits(M, N, K)
    ws = torch.empty(sp * M * N, device=gpu) if epi == 7 else None
    C_.gemm2(A, B, C, 1, 1, epi, None, None, None, 0.0, 0, sp, ws, None)
    _check(C, C0 + A.float().t() @ B.float(), acc=A.float().abs().t() @ B.float().abs() + C0.abs(), fp32=True)


@pytest.mark.parametrize("M,N,K", [(50432, 1024, 4928), (2304, 768, 512), (768, 256, 320)])
@pytest.mark.parametrize("small", ["0", "1"])
def test_gemm2_tt_one_split_accumulates_in_place(gpu, monkeypatch, M, N, K, small):
    """TT weight gradient with one K-split (the tied MLM decoder table: Vp x H over the masked tokens): C += Aᵀ·B in
    place, each element written by its one owner (no fp32 atomics), on the 256 and the 128 tile kernels; against the
    fp32 reference and the atomic-epilogue path (HSD_G2_TT_ATOMIC=1)."""
    monkeypatch.setenv("HSD_G2_SMALL_TT", small)
    torch.manual_seed(13)
    C_ = _C()
    A, B = _mk((K, M), gpu), _mk((K, N), gpu)
    C0 = torch.randn(M, N, device=gpu)
    outs = []
    for atomic in ("0", "1"):
        monkeypatch.setenv("HSD_G2_TT_ATOMIC", atomic)
        C = C0.clone()
        ws = torch.empty(M * N, device=gpu)  # the binding's workspace contract (unused with one split)
        C_.gemm2(A, B, C, 1, 1, 7, None, None, None, 0.0, 0, 1, ws, None)
        torch.cuda.synchronize()
        outs.append(C)
    ref = C0 + A.float().t() @ B.float()
    acc = A.float().abs().t() @ B.float().abs() + C0.abs()
    _check(outs[0], ref, acc=acc, fp32=True)
    torch.testing.assert_close(outs[0], outs[1], rtol=0, atol=0)  # one owner per element: same sum either way


@pytest.mark.parametrize("sync", [0, 1, 4, 5, 6, 7])
@pytest.mark.parametrize("M,N,K", [(1000, 960, 192), (768, 3072, 512), (2048, 768, 3072)])
def test_gemm2_schedules(gpu, monkeypatch, sync, M, N, K):
    """Every main-loop schedule (HSD_G2_SYNC: 8-phase, one-barrier, staggered 4 / 5) gives the fp32-reference
    NT product (bias epilogue) and, where the shape tiles, the TT weight gradient (tokens = M)."""
    monkeypatch.setenv("HSD_G2_SYNC", str(sync))
    torch.manual_seed(21)
    C_ = _C()
    A, B, bias = _mk((M, K), gpu), _mk((N, K), gpu, 0.1), _mk((N,), gpu)
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    C_.gemm2(A, B, C, 0, 0, 1, bias, None, None, 0.0, 0, 1, None, None)
    _check(C, A.float() @ B.float().t() + bias.float(), acc=_absmm(A, B, 0, 0))
    if K % 256 == 0 and M % 64 == 0:
        dy = _mk((M, N), gpu)
        G0 = torch.randn(N, K, device=gpu)
        G = G0.clone()
        sp = C_.gemm2_splits(N, K, M)
        ws = torch.empty(sp * N * K, device=gpu)
        C_.gemm2(dy, A, G, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)
        _check(G, G0 + dy.float().t() @ A.float(), acc=dy.float().abs().t() @ A.float().abs() + G0.abs(), fp32=True)


def test_gemm2_dgelu_fused_dbias(gpu):
    torch.manual_seed(13)
    C_ = _C()
    M, N, K = 1024, 3072, 768
    A, B, pre = _mk((M, K), gpu), _mk((N, K), gpu, 0.1), _mk((M, N), gpu)
    C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    db = torch.full((N,), 0.5, device=gpu)
    C_.gemm2(A, B, C, 0, 0, 5, None, pre, None, 0.0, 0, 1, None, db)
    a32, gg = A.float() @ B.float().t(), _gelu_grad(pre.float())
    r = a32.bfloat16().float() * gg
    _check(C, r, mag=2 * a32.abs() * gg.abs() + r.abs(), acc=2 * _absmm(A, B, 0, 0))
    _check(db, 0.5 + C.float().sum(0), acc=0.5 + C.float().abs().sum(0), fp32=True)


def test_gemm2_gelu_derivative_and_mul_epilogues(gpu):
    """E2_BIAS_GELU_D (C = gelu'(y), C2 = gelu(y)) and E2_MUL (C = bf16(acc) * aux, + fused column sums)."""
    torch.manual_seed(14)
    C_ = _C()
    M, N, K = 512, 3072, 768
    A, B, bias = _mk((M, K), gpu), _mk((N, K), gpu, 0.1), _mk((N,), gpu)
    D = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    G = torch.empty_like(D)
    C_.gemm2(A, B, D, 0, 0, 8, bias, None, G, 0.0, 0, 1, None, None)
    y = (A.float() @ B.float().t() + bias.float()).bfloat16().float()
    g, d = torch.nn.functional.gelu(y), _gelu_grad(y)
    am = _absmm(A, B, 0, 0)  # the kernel's y may differ from torch's by fp32 accumulation order before rounding
    _check(G, g, mag=2 * y.abs() + g.abs(), acc=2 * am)
    _check(D, d, mag=y.abs() + d.abs(), acc=am)
    dy, W = _mk((M, 768), gpu), _mk((N, 768), gpu, 0.1)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    db = torch.zeros(N, device=gpu)
    C_.gemm2(dy, W, out, 0, 0, 9, None, D, None, 0.0, 0, 1, None, db)
    a32 = dy.float() @ W.float().t()
    r = a32.bfloat16().float() * D.float()
    _check(out, r, mag=2 * a32.abs() * D.float().abs() + r.abs(), acc=2 * _absmm(dy, W, 0, 0))
    _check(db, out.float().sum(0), acc=out.float().abs().sum(0), fp32=True)


@pytest.mark.parametrize("small", ["0", "1"])
@pytest.mark.parametrize("M,N,K,splits", [(512, 768, 1024, 4), (300, 512, 3072, 3), (4096, 1024, 4096, 0),
                                          (128, 768, 3072, 0), (128, 3072, 768, 0)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 8, 9])
def test_gemm2_nt_splitk_matches_one_pass(gpu, monkeypatch, M, N, K, splits, epi, small):
    """Split-K NT (fp32 slabs + reduce-and-epilogue pass) == the one-pass fused epilogue, for every epilogue kind
    (same dropout sites, same fused bias-gradient column sums), up to the fp32 order of the K-split sums."""
    torch.manual_seed(5 + epi)
    C_ = _C()
    # split-K slabs from the 256 x 256 kernel (small = "0") or the 128 x 128 kernel ("1": serving batches)
    monkeypatch.setenv("HSD_G2_SMALL", small)
    if splits == 0 and (small == "0") == (M != 128):
        assert C_.gemm2_nt_splits(M, N, K) > 1  # small tile grids are split automatically
    A, B = _mk((M, K), gpu), _mk((N, K), gpu, 0.05)
    bias = _mk((N,), gpu)
    aux = _mk((M, N), gpu) if epi != 9 else torch.rand(M, N, device=gpu).bfloat16()
    two = epi in (2, 8)
    p = 0.1 if epi == 3 else 0.0
    outs = []
    for sp in (1, splits):
        C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        C2 = torch.empty_like(C) if two else None
        db = torch.zeros(N, device=gpu) if epi in (5, 9) and N % 256 == 0 else None
        C_.gemm2(A, B, C, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None,
                 C2, p, 77, sp, None, db)
        outs.append((C.float(), C2.float() if two else None, db))
    (c1, c21, d1), (cs, c2s, ds) = outs
    # the split sums differ from the one-pass sum in fp32 order only: one ulp of every rounded intermediate
    y = (A.float() @ B.float().t() + (bias.float() if epi in (1, 2, 3, 8) else 0.0)).abs()
    ax = aux.float().abs()
    mag = 2 * y * (1 + ax) + ax + c1.abs()
    _check(cs, c1, mag=mag, acc=2 * _absmm(A, B, 0, 0))
    if two:
        _check(c2s, c21, mag=mag + c21.abs())
    if d1 is not None:
        torch.testing.assert_close(ds, d1, rtol=2e-2, atol=1e-2 * float(d1.abs().max()) + 1e-3)


@pytest.mark.parametrize("stages", [2, 3, 4])
@pytest.mark.parametrize("M,N,K", [(300, 512, 1024), (4096, 1024, 1024), (128, 768, 3072)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 8, 9])
def test_gemm2_small_tiles_match_256_tiles(gpu, monkeypatch, M, N, K, epi, stages):
    """gemm2s (128 x 128 tiles, for grids 256 x 256 tiles leave idle) == gemm2 bit for bit on every epilogue (same
    K order per element, same dropout sites); fused bias-gradient column sums to fp32 rounding."""
    torch.manual_seed(3 + epi)
    C_ = _C()
    A, B = _mk((M, K), gpu), _mk((N, K), gpu, 0.05)
    bias = _mk((N,), gpu)
    aux = _mk((M, N), gpu) if epi != 9 else torch.rand(M, N, device=gpu).bfloat16()
    two = epi in (2, 8)
    outs = []
    monkeypatch.setenv("HSD_G2S_STAGES", str(stages))
    # the 4-wave kernel (the 8-wave in-workgroup K-split sums the K halves in another order:
    # test_gemm2_small_tiles_kw2_matches_kw1)
    monkeypatch.setenv("HSD_G2S_KW", "1")
    for small in ("0", "1"):
        monkeypatch.setenv("HSD_G2_SMALL", small)
        monkeypatch.setenv("HSD_G2_SPLITK", "1")
        C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        C2 = torch.empty_like(C) if two else None
        db = torch.zeros(N, device=gpu) if epi in (5, 9) and N % 256 == 0 else None
        C_.gemm2(A, B, C, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None,
                 C2, 0.1 if epi == 3 else 0.0, 77, 0, None, db)
        torch.cuda.synchronize()
        outs.append((C, C2, db))
    (c0, c20, d0), (c1, c21, d1) = outs
    assert torch.equal(c0, c1)
    if two:
        assert torch.equal(c20, c21)
    if d0 is not None:
        torch.testing.assert_close(d1, d0, rtol=1e-4, atol=1e-4 * float(d0.abs().max()) + 1e-6)


@pytest.mark.parametrize("M,N,K", [(4096, 1024, 1024), (300, 512, 1024), (128, 768, 3072), (4096, 1024, 4096)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 8, 9])
@pytest.mark.parametrize("lb", [0, 1])
def test_gemm2_small_tiles_kw2_matches_kw1(gpu, monkeypatch, M, N, K, epi, lb):
    """gemm2s with the in-workgroup K-split (HSD_G2S_KW=2: 8 waves, wave groups on the two halves of every K-tile,
    partial tiles summed through LDS) vs the 4-wave kernel: same epilogues and dropout sites, the fp32 sum in another
    order (one bf16 ulp of the rounded intermediates), for k-contiguous and k-strided (W read directly) B."""
    torch.manual_seed(7 + epi)
    C_ = _C()
    A = _mk((M, K), gpu)
    W = _mk((N, K), gpu, 0.05)  # lb 0: B = W [N][K]; lb 1: B = Wᵀ stored as [K][N]
    B = W if lb == 0 else W.t().contiguous()
    bias = _mk((N,), gpu)
    aux = _mk((M, N), gpu) if epi != 9 else torch.rand(M, N, device=gpu).bfloat16()
    two = epi in (2, 8)
    if lb == 1 and not C_.gemm2_supported(0, 1, epi, M, N, K):
        pytest.skip("layout (0, 1) epilogue not supported at this shape")
    outs = []
    monkeypatch.setenv("HSD_G2S_STAGES", "3")
    monkeypatch.setenv("HSD_G2_SMALL", "1")
    monkeypatch.setenv("HSD_G2_SPLITK", "1")
    for kw in ("1", "2"):
        monkeypatch.setenv("HSD_G2S_KW", kw)
        C_.refresh_env()
        C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        C2 = torch.empty_like(C) if two else None
        db = torch.zeros(N, device=gpu) if epi in (5, 9) and N % 256 == 0 else None
        C_.gemm2(A, B, C, 0, lb, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None,
                 C2, 0.1 if epi == 3 else 0.0, 77, 0, None, db)
        torch.cuda.synchronize()
        outs.append((C, C2, db))
    monkeypatch.delenv("HSD_G2S_KW")
    C_.refresh_env()
    (c1, c21, d1), (c2, c22, d2) = outs
    y = A.float() @ W.float().t() + (bias.float() if epi in (1, 2, 3, 8) else 0.0)
    mag = c1.float().abs() + y.abs() + (aux.float().abs() if epi in (3, 4) else 0.0)
    _check(c2, c1.float(), mag=mag, acc=2 * _absmm(A, W, 0, 0) * (aux.float().abs() + 1 if epi in (5, 9) else 1))
    if two:
        _check(c22, c21.float(), mag=c21.float().abs() + y.abs(), acc=2 * _absmm(A, W, 0, 0))
    if d1 is not None:
        torch.testing.assert_close(d2, d1, rtol=2e-2, atol=1e-2 * float(d1.abs().max()) + 1e-3)


@pytest.mark.parametrize("stages,kw", [(2, 1), (3, 1), (3, 2), (4, 1)])
@pytest.mark.parametrize("M,N,K,splits", [(1024, 1024, 4096, 0), (1024, 1024, 4096, 1), (3072, 1024, 4096, 0),
                                          (1000, 768, 512, 0), (1024, 4096, 128, 0), (200, 384, 1024, 3)])
def test_gemm2_small_tt_wgrad(gpu, monkeypatch, M, N, K, splits, stages, kw):
    """gemm2s TT (128 x 128 tiles): weight gradient C += Aᵀ·B in fp32, one split accumulating in place or K-splits
    into slabs + reduce, every stage depth and both workgroup shapes (kw 2: in-workgroup K-split), against the fp32
    reference."""
    monkeypatch.setenv("HSD_G2_SMALL_TT", "1")
    monkeypatch.setenv("HSD_G2S_STAGES", str(stages))
    monkeypatch.setenv("HSD_G2S_KW", str(kw))
    torch.manual_seed(31)
    C_ = _C()
    A, B = _mk((K, M), gpu), _mk((K, N), gpu)
    C0 = torch.randn(M, N, device=gpu)
    C = C0.clone()
    sp = splits or C_.gemm2_splits(M, N, K)
    ws = torch.empty(sp * M * N, device=gpu)
    C_.gemm2(A, B, C, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)
    _check(C, C0 + A.float().t() @ B.float(), acc=A.float().abs().t() @ B.float().abs() + C0.abs(), fp32=True)




@pytest.mark.parametrize("M,N,K", [(4096, 1024, 1024), (4096, 4096, 1024), (4096, 1024, 4096), (1000, 768, 3072),
                                   (131072 // 16, 768, 3072), (64, 1024, 1024), (1024, 1024, 16384)])
@pytest.mark.parametrize("epi", [0, 4, 5, 9])
def test_gemm2_dgrad_reading_w_directly_matches_stored_wt(gpu, M, N, K, epi):
    """The dgrad on W [K][N] as the NT kernel's k-strided B operand (layout (0, 1): small steps keep no Wᵀ copy)
    equals the dgrad on the stored Wᵀ [N][K] (layout (0, 0)) bit for bit: same fragments, same K order. Shapes cover
    the 128 x 128 kernel, the 256 x 256 kernel, split-K slabs and a fused bias-gradient column sum."""
    torch.manual_seed(31 + epi)
    C_ = _C()
    dy, w = _mk((M, K), gpu), _mk((K, N), gpu, 0.05)
    aux = _mk((M, N), gpu) if epi != 9 else torch.rand(M, N, device=gpu).bfloat16()
    outs = []
    for la_lb, B in (((0, 0), w.t().contiguous()), ((0, 1), w)):
        C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        db = torch.zeros(N, device=gpu) if epi in (5, 9) and N % 256 == 0 else None
        if not C_.gemm2_supported(la_lb[0], la_lb[1], epi, M, N, K):
            pytest.skip("shape not tiled")
        C_.gemm2(dy, B, C, la_lb[0], la_lb[1], epi, None, aux if epi in (4, 5, 9) else None, None, 0.0, 0, 0, None, db)
        torch.cuda.synchronize()
        outs.append((C, db))
    (c0, d0), (c1, d1) = outs
    assert torch.equal(c0, c1)
    if d0 is not None:
        torch.testing.assert_close(d1, d0, rtol=1e-4, atol=1e-4 * float(d0.abs().max()) + 1e-6)
    ref = dy.float() @ w.float()
    if epi == 0:
        _check(c1, ref, acc=dy.float().abs() @ w.float().abs())


@pytest.mark.parametrize("M,N,K", [(32768, 768, 256), (8292, 3072, 512), (20000, 960, 128), (65536, 2304, 64)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 8, 9])
def test_gemm2_persistent_matches_one_shot(gpu, monkeypatch, M, N, K, epi):
    """Persistent NT kernel (gemm2pk: one workgroup per CU walking tiles, next tile's DMA under the epilogue) ==
    the one-shot gemm2 kernel bit for bit on every bf16 epilogue (same main loop, same dropout sites); fused
    bias-gradient column sums to fp32 rounding (atomic order). Shapes: >1 round of tiles, BN 256 and 192, M edges."""
    torch.manual_seed(41 + epi)
    C_ = _C()
    A, B = _mk((M, K), gpu), _mk((N, K), gpu, 0.05)
    bias = _mk((N,), gpu)
    aux = _mk((M, N), gpu) if epi != 9 else torch.rand(M, N, device=gpu).bfloat16()
    two = epi in (2, 8)
    outs = []
    monkeypatch.setenv("HSD_G2_SPLITK", "1")
    for persist in ("0", "1"):
        monkeypatch.setenv("HSD_G2_PERSIST", persist)
        C = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        C2 = torch.empty_like(C) if two else None
        db = torch.zeros(N, device=gpu) if epi in (5, 9) and N % 256 == 0 else None
        C_.gemm2(A, B, C, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None, aux if epi in (3, 4, 5, 9) else None,
                 C2, 0.1 if epi == 3 else 0.0, 77, 0, None, db)
        torch.cuda.synchronize()
        outs.append((C, C2, db))
    (c0, c20, d0), (c1, c21, d1) = outs
    assert torch.equal(c0, c1)
    if two:
        assert torch.equal(c20, c21)
    if d0 is not None:
        torch.testing.assert_close(d1, d0, rtol=1e-4, atol=1e-4 * float(d0.abs().max()) + 1e-6)
    if epi == 0:
        _check(c1, A.float() @ B.float().t(), acc=_absmm(A, B, 0, 0))


@pytest.mark.parametrize("path", ["pk", "oneshot", "small", "splitk"])
@pytest.mark.parametrize("lb", [0, 1])
@pytest.mark.parametrize("B_,S,heads,K", [(16, 512, 12, 768), (2, 512, 16, 1024), (3, 384, 16, 4096)])
def test_gemm2_row_dot_epilogue_feeds_attention_backward(gpu, monkeypatch, path, lb, B_, S, heads, K):
    """E2_STORE_RDOT (the out-projection dgrad also writing the streaming attention backward's delta rows): dx is
    bit-identical to the plain store epilogue on every kernel path (persistent, one-shot, 128-tile, split-K), the rows
    are bit-identical to the attention's own delta pass (one shared dot8_bf16 + sum8_dpp), and the backward fed those
    rows (delta_ready) gives the same dqkv bits as the one that computes them itself."""
    if path == "pk" and lb == 1:
        pytest.skip("the persistent kernel reads a stored Wᵀ (lb = 0) only")
    torch.manual_seed(11 + K)
    C_ = _C()
    monkeypatch.setenv("HSD_G2_PERSIST", "1" if path == "pk" else "0")
    monkeypatch.setenv("HSD_G2_SMALL", "1" if path == "small" else "0")
    monkeypatch.setenv("HSD_G2_SPLITK", "3" if path == "splitk" else "1")
    H = heads * 64
    T = B_ * S
    dy = _mk((T, K), gpu)
    W = _mk((K, H), gpu, 0.05)            # B[K][N] (lb = 1)
    Bop = W if lb == 1 else W.t().contiguous()  # Wᵀ [N][K] (lb = 0)
    qkv = _mk((T, 3 * H), gpu)
    o = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    lse = torch.empty(B_ * heads * S, device=gpu)
    C_.attn_fwd(qkv, None, o, lse, B_, S, heads, 0.1, 99, None)
    dx0 = torch.empty(T, H, device=gpu, dtype=torch.bfloat16)
    C_.gemm2(dy, Bop, dx0, 0, lb, 0, None, None, None, 0.0, 0, 0, None, None)
    dx1 = torch.empty_like(dx0)
    rd = torch.full((B_ * heads * S,), float("nan"), device=gpu)
    C_.gemm2(dy, Bop, dx1, 0, lb, 10, None, o, None, 0.0, 0, 0, None, None, rd, S)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)
    ref = (dx0.float() * o.float()).view(B_, S, heads, 64).sum(-1).permute(0, 2, 1).reshape(-1)
    torch.testing.assert_close(rd, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
    outs = []
    for ready in (False, True):
        ws = rd.clone() if ready else torch.empty_like(rd)
        dqkv = torch.empty_like(qkv)
        db = torch.zeros(3 * H, device=gpu)
        C_.attn_bwd(qkv, None, o, dx0, lse, dqkv, ws, B_, S, heads, 0.1, 99, db, None, ready)
        torch.cuda.synchronize()
        outs.append((ws, dqkv, db))
    (ws0, dq0, db0), (ws1, dq1, db1) = outs
    assert torch.equal(ws0, rd)  # the attention's own delta pass wrote the same bits
    assert torch.equal(dq0, dq1)
    torch.testing.assert_close(db1, db0, rtol=1e-5, atol=1e-5 * float(db0.abs().max()) + 1e-6)
