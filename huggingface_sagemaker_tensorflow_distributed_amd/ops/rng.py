"""Counter-based dropout RNG shared bit-for-bit by the torch reference path and the HIP kernels.

Why counter-based: dropout masks are never stored; the backward kernels regenerate the mask of
element ``e`` from ``(seed, e)``. The reference's TF dropout draws from a
stateful Philox stream; we need the same *distribution* (Bernoulli keep with prob ``1-p``, scale
``1/(1-p)``) and determinism between forward and backward, not TF's exact bit stream.

Definition (mirrored in ``csrc/kernels/common.h::dropout_bits``):

* the site's 64-bit seed is mixed once into a 32-bit key ``k = mix32(seed_lo ^ mix32(seed_hi))``
  (``mix32`` = lowbias32, Wellons);
* element pair ``j`` (elements ``2j`` and ``2j+1`` of the flattened site tensor) draws
  ``h = mix32(j ^ k)`` — one round per pair: the attention kernels hash every (query, key) pair;
* element ``2j`` keeps iff ``(h & 0xFFFF) >= thr``; element ``2j+1`` keeps iff ``(h >> 16) >= thr``;
* ``thr = round(p * 65536)``.
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF
_C1 = 0x7FEB352D
_C2 = 0x846CA68B


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


def threshold(p: float) -> int:
    return int(round(p * 65536.0))


def keep_mask(seed: int, numel: int, p: float, device=None) -> torch.Tensor:
    """Boolean keep mask of ``numel`` elements for a dropout site with 64-bit ``seed``."""
    seed_lo = seed & M32
    seed_hi = (seed >> 32) & M32
    key = site_key(seed_lo, seed_hi)
    npairs = (numel + 1) // 2
    j = torch.arange(npairs, dtype=torch.int64, device=device)
    h = mix32(j ^ key)
    lo = h & 0xFFFF
    hi = h >> 16
    bits = torch.stack([lo, hi], dim=1).reshape(-1)[:numel]
    return bits >= threshold(p)


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
