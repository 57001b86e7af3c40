"""Dropout mask definition (ops/rng.py, csrc/kernels/common.h): the Python reference equals the kernels' host-side
evaluation bit for bit, and the masks have the statistics of independent Bernoulli(1 - p) draws (SURVEY.md §2.10 N.6;
reference: Keras dropout p = 0.1 in every BERT layer, scripts/train.py:117)."""
import numpy as np
import pytest
import torch

from huggingface_sagemaker_tensorflow_distributed_amd.ops import rng


def _np_bits(key, rows, cps):
    """Vectorised numpy copy of rng.pair_bits (uint64 arithmetic, masked to 32 bits)."""
    m = np.uint64(0xFFFFFFFF)

    def mix(x):
        x = x & m
        x ^= x >> np.uint64(16)
        x = (x * np.uint64(rng._C1)) & m
        x ^= x >> np.uint64(15)
        x = (x * np.uint64(rng._C2)) & m
        x ^= x >> np.uint64(16)
        return x

    col = np.zeros_like(cps)
    for i in range(32):
        if (rng.DROP_C >> i) & 1:
            col ^= (cps << np.uint64(i)) & m
    y = ((mix(rows ^ np.uint64(key)) ^ col) * np.uint64(rng.DROP_M)) & m
    return y ^ (y >> np.uint64(16))


def test_python_matches_kernel_definition():
    from huggingface_sagemaker_tensorflow_distributed_amd.ops._ext import load

    C = load()
    g = np.random.default_rng(0)
    for seed in (0, 1, 0xDEADBEEF12345678, (1 << 63) + 12345):
        key = rng.site_key(seed & rng.M32, (seed >> 32) & rng.M32)
        rows = g.integers(0, 1 << 31, 64)
        cps = g.integers(0, 1 << 12, 64)
        ref = rng.pair_bits(key, torch.from_numpy(rows), torch.from_numpy(cps))
        s64 = seed - (1 << 64) if seed >= 1 << 63 else seed
        for r, c, v in zip(rows.tolist(), cps.tolist(), ref.tolist()):
            assert C.dropout_pair_bits(s64, r, c) == v
        assert np.array_equal(_np_bits(key, rows.astype(np.uint64), cps.astype(np.uint64)), ref.numpy())


def test_column_word_is_linear():
    """Kernels fold lane / tile offsets with XORs: C(a ^ b) == C(a) ^ C(b)."""
    g = np.random.default_rng(1)
    for a, b in g.integers(0, 1 << 16, (200, 2)).tolist():
        assert rng.drop_col_int(a ^ b) == rng.drop_col_int(a) ^ rng.drop_col_int(b)


def test_keep_mask_layout():
    """keep_mask views the site as [rows, W]: element (r, 2cp) takes the low 16 bits of pair (r, cp), (r, 2cp+1) the
    high 16; the last dimension is the row width."""
    seed, p = 0x1234_5678_9ABC, 0.3
    m = rng.keep_mask(seed, (3, 5, 8), p)
    key = rng.site_key(seed & rng.M32, seed >> 32)
    thr = rng.threshold(p)
    for r in range(15):
        for c in range(8):
            h = int(rng.pair_bits(key, torch.tensor(r), torch.tensor(c // 2)))
            half = (h >> 16) if c & 1 else (h & 0xFFFF)
            assert bool(m.view(15, 8)[r, c]) == (half >= thr)
    with pytest.raises(TypeError):
        rng.keep_mask(seed, 120, p)


def test_keep_rate_over_1e8_draws():
    """Keep rate within 3 sigma of 1 - thr/65536 over 1e8 draws (bert-base-like [rows, 768] sites, several keys)."""
    p = 0.1
    thr = rng.threshold(p)
    q = 1.0 - thr / 65536.0
    n = kept = 0
    W2 = 384  # column pairs of a 768-wide row
    cps = np.arange(W2, dtype=np.uint64)[None, :]
    rows_per_chunk = 16384
    for chunk in range(8):
        key = rng.site_key(0x9E37 * (chunk + 1), chunk)
        rows = np.arange(rows_per_chunk, dtype=np.uint64)[:, None] + np.uint64(chunk * 1_000_003)
        h = _np_bits(key, rows, cps)
        kept += int(((h & np.uint64(0xFFFF)) >= thr).sum()) + int(((h >> np.uint64(16)) >= thr).sum())
        n += 2 * h.size
    assert n >= 1e8
    rate = kept / n
    sigma = np.sqrt(q * (1 - q) / n)
    assert abs(rate - q) <= 3 * sigma, (rate, q, sigma)


def _corr(a, b):
    a = a.astype(np.float64).ravel() - a.mean()
    b = b.astype(np.float64).ravel() - b.mean()
    return float((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean()))


@pytest.mark.parametrize("W", [128, 512, 768])
def test_no_neighbour_correlation(W):
    """No correlation between neighbouring elements along rows, columns, the two halves of a pair, diagonals and
    power-of-two strides (|z| < 5 for each of ~20 statistics), and 2x2 block patterns consistent with independence."""
    p = 0.1
    thr = rng.threshold(p)
    rows = 8192 if W <= 512 else 4096
    key = rng.site_key(0xABCDEF, 0x13579)
    h = _np_bits(key, np.arange(rows, dtype=np.uint64)[:, None], np.arange(W // 2, dtype=np.uint64)[None, :])
    k = np.empty((rows, W), dtype=bool)
    k[:, 0::2] = (h & np.uint64(0xFFFF)) >= thr
    k[:, 1::2] = (h >> np.uint64(16)) >= thr
    sig = 1.0 / np.sqrt(k.size)
    tests = {"halves": (k[:, 0::2], k[:, 1::2]), "col+1": (k[:, :-1], k[:, 1:]), "col+2": (k[:, :-2], k[:, 2:]),
             "row+1": (k[:-1], k[1:]), "diag": (k[:-1, :-1], k[1:, 1:]), "anti": (k[:-1, 1:], k[1:, :-1])}
    for s in (4, 8, 16, 32, 64):
        tests[f"col+{s}"] = (k[:, :-s], k[:, s:])
        tests[f"row+{s}"] = (k[:-s], k[s:])
    for name, (a, b) in tests.items():
        z = _corr(a, b) / sig
        assert abs(z) < 5.0, (name, z)
    # 2x2 blocks over (rows r, r+1) x (columns 2j, 2j+2): 16 patterns, chi-square with 15 dof (p < 1e-4 -> 44.3)
    a, b, c, d = k[0::2, 0:-2:4], k[0::2, 2::4], k[1::2, 0:-2:4], k[1::2, 2::4]
    nn = min(a.shape[1], b.shape[1])
    pat = (a[:, :nn] + 2 * b[:, :nn] + 4 * c[:, :nn] + 8 * d[:, :nn].astype(np.int64)).ravel()
    obs = np.bincount(pat.astype(np.int64), minlength=16).astype(np.float64)
    q = 1.0 - thr / 65536.0
    ones = np.array([bin(i).count("1") for i in range(16)])
    exp = pat.size * q ** ones * (1 - q) ** (4 - ones)
    chi2 = float(((obs - exp) ** 2 / exp).sum())
    assert chi2 < 44.3, chi2


@pytest.mark.parametrize("W", [128, 1024])
def test_cross_row_twin_masks_occur_at_the_random_function_rate(W):
    """because C is GF(2)-linear, rows r1, r2 whose row words satisfy R(r1) ^ R(r2) = C(d) for some
    0 < d < W/2 have masks that are the same bits with the column pairs permuted (bits(r1, c) == bits(r2, c ^ d) for
    every c). This is the documented trade-off of the one-XOR-per-pair column word (common.h): R = lowbias32 of the
    row is a bijection, so each row pair hits one of the W/2 - 1 forbidden differences with probability
    (W/2 - 1) / 2^32 -- the same rate as for a random function, no structure beyond it. A twin keeps the same number
    of elements and a data-independent permutation of them. Here: the count over 2^17 rows (the bert-base B = 1024
    S = 128 attention site's row count) matches n^2/2 x (W/2 - 1) / 2^32 within 5 sigma (Poisson), and every found
    pair really is a permuted copy."""
    n = 1 << 17
    key = rng.site_key(0x1234567, 0x89ABCDE)
    R = rng.mix32(torch.arange(n, dtype=torch.int64) ^ key).numpy().astype(np.uint32)
    order = np.argsort(R)
    Rs = R[order]
    found, example = 0, None
    for d in range(1, W // 2):
        t = (R ^ np.uint32(rng.drop_col_int(d))).astype(np.uint32)
        pos = np.searchsorted(Rs, t)
        pos[pos == n] = 0
        hit = Rs[pos] == t
        found += int(hit.sum())
        if example is None and hit.any():
            i = int(np.nonzero(hit)[0][0])
            example = (i, int(order[pos[i]]), d)
    found //= 2  # each twin pair is seen from both rows
    expect = n * n / 2 * (W // 2 - 1) / 2.0 ** 32
    assert abs(found - expect) <= 5 * expect ** 0.5 + 1, (found, expect)
    if example is not None:
        r1, r2, d = example
        cps = torch.arange(W // 2, dtype=torch.int64)
        b1 = rng.pair_bits(key, torch.full_like(cps, r1), cps)
        b2 = rng.pair_bits(key, torch.full_like(cps, r2), cps ^ d)
        assert torch.equal(b1, b2)
