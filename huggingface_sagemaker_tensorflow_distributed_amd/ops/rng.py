"""Counter-based dropout RNG shared bit-for-bit by the torch reference path and the HIP kernels.

Why counter-based: dropout masks are never stored; the backward kernels regenerate the mask of
element ``e`` from ``(seed, e)``. The reference's TF dropout draws from a
stateful Philox stream; we need the same *distribution* (Bernoulli keep with prob ``1-p``, scale
``1/(1-p)``) and determinism between forward and backward, not TF's exact bit stream.

Definition (mirrored in ``csrc/kernels/common.h``, dropout mask section). A dropout site of shape ``[..., W]`` is
viewed as ``[rows, W]``; element ``(r, c)`` belongs to column pair ``cp = c // 2`` of row ``r``:

* the site's 64-bit seed is mixed once into a 32-bit key ``k = mix32(seed_lo ^ mix32(seed_hi))``
  (``mix32`` = lowbias32, Wellons);
* the row word ``R(r) = mix32(r ^ k)`` (one full hash per ROW: kernels hold it in a register across the row);
* the column word ``C(cp) = clmul32(cp, 0x6D2B79F5)`` (carry-less product: GF(2)-linear, so kernels fold their
  lane / tile offsets into one register with XORs and every register offset is a compile-time constant);
* the pair's bits ``h = y ^ (y >> 16)`` with ``y = (R(r) ^ C(cp)) * 0x9E3779B1 mod 2^32``;
* column ``2cp`` keeps iff ``(h & 0xFFFF) >= thr``; column ``2cp+1`` keeps iff ``(h >> 16) >= thr``;
  ``thr = round(p * 65536)``.

Per element pair a kernel spends one XOR, one multiply and one XOR (round 4: two lowbias32 multiplies, three
xor-shifts and the pair arithmetic per pair). Statistics: ``tests/test_rng.py`` (keep rate over 1e8 draws, neighbour
correlations, 2x2 block patterns), ``tools/rng_quality.py`` (the candidate screen).
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF
_C1 = 0x7FEB352D
_C2 = 0x846CA68B
DROP_C = 0x6D2B79F5
DROP_M = 0x9E3779B1


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    # (x * c) mod 2^32 without signed int64 overflow: split c into 16-bit halves.
    lo = c & 0xFFFF
    hi = c >> 16
    return (x * lo + (((x * hi) & 0xFFFF) << 16)) & M32


def mix32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = _mul32(x, _C1)
    x = x ^ (x >> 15)
    x = _mul32(x, _C2)
    x = x ^ (x >> 16)
    return x


def mix32_int(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * _C1) & M32
    x ^= x >> 15
    x = (x * _C2) & M32
    x ^= x >> 16
    return x


def site_key(seed_lo: int, seed_hi: int) -> int:
    """32-bit key of a dropout site (``common.h::dropout_key``)."""
    return mix32_int((seed_lo & M32) ^ mix32_int(seed_hi & M32))


def drop_col(cp: torch.Tensor) -> torch.Tensor:
    """``C(cp)``: carry-less product of the column-pair index with DROP_C, mod 2^32."""
    out = torch.zeros_like(cp)
    for i in range(32):
        if (DROP_C >> i) & 1:
            out = out ^ ((cp << i) & M32)
    return out


def drop_col_int(cp: int) -> int:
    o = 0
    for i in range(32):
        if (DROP_C >> i) & 1:
            o ^= (cp << i) & M32
    return o


def drop_fin(x: torch.Tensor) -> torch.Tensor:
    y = _mul32(x, DROP_M)
    return y ^ (y >> 16)


def threshold(p: float) -> int:
    return int(round(p * 65536.0))


def pair_bits(key: int, rows: torch.Tensor, cps: torch.Tensor) -> torch.Tensor:
    """32 mask bits of column pair ``cps`` of row ``rows`` (int64 tensors, broadcast) for site key ``key``."""
    return drop_fin(mix32((rows & M32) ^ key) ^ drop_col(cps & M32))


def keep_mask(seed: int, shape, p: float, device=None) -> torch.Tensor:
    """Boolean keep mask of a dropout site of ``shape`` (a tuple / torch.Size; the last dimension is the row width W)
    with 64-bit ``seed``."""
    if isinstance(shape, int):
        raise TypeError("keep_mask: pass the site's shape (its last dimension is the mask's row width), not numel")
    shape = tuple(int(d) for d in shape)
    W = shape[-1] if shape else 1
    numel = 1
    for d in shape:
        numel *= d
    rows = numel // W if W else 0
    key = site_key(seed & M32, (seed >> 32) & M32)
    r = torch.arange(rows, dtype=torch.int64, device=device).unsqueeze(1)
    cp = torch.arange((W + 1) // 2, dtype=torch.int64, device=device).unsqueeze(0)
    h = pair_bits(key, r, cp)
    bits = torch.stack([h & 0xFFFF, h >> 16], dim=2).reshape(rows, -1)[:, :W]
    return (bits >= threshold(p)).reshape(shape)


class DropoutSeeds:
    """Hands out one 64-bit seed per dropout call site per step.

    Seeds are derived deterministically from ``(base_seed, step, call_index)`` so a replayed step
    (e.g. re-running forward for a check) regenerates identical masks, and data-parallel ranks can
    choose to share or decorrelate masks (``rank`` is mixed in by default, like independent TF
    replicas).
    """

    def __init__(self, base_seed: int = 0, rank: int = 0):
        self.base_seed = int(base_seed)
        self.rank = int(rank)
        self.step = 0
        self.calls = 0

    def new_step(self, step: int | None = None) -> None:
        self.step = self.step + 1 if step is None else int(step)
        self.calls = 0

    def next(self) -> int:
        a = mix32_int(self.base_seed ^ 0x9E3779B9)
        b = mix32_int(a ^ (self.step * 0x85EBCA6B + self.rank * 0xC2B2AE35))
        c = mix32_int(b ^ (self.calls * 0x27D4EB2F + 0x165667B1))
        d = mix32_int(c ^ a ^ 0x5BD1E995)
        self.calls += 1
        return (c << 32) | d
