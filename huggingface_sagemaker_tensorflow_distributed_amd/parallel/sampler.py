"""Rank sharding of the dataset (SURVEY.md §2.8 Q3 fix).

The reference batches the full dataset on every rank (``scripts/train.py:84-86``: no
``.shard(hvd.size(), hvd.rank())``), so N ranks train on N identical copies. We shard: rank ``r``
takes examples ``r, r+N, r+2N, ...`` of a (optionally shuffled, seed-shared) permutation, the tail is
dropped so every rank runs the same number of steps (collectives stay matched).

Evaluation must score every example exactly once, as ``model.evaluate`` does on the reference's unsharded
test set (``scripts/train.py:170``), including the last partial batch. ``drop_last=False,
mark_padding=True`` pads the permutation to a multiple of N with repeats encoded as ``-(index + 1)``; the
loader turns them into ignored rows (label -100) that the metric meter does not count.
"""
from __future__ import annotations

from typing import Iterator, List, Optional

import torch


class ShardSampler:
    def __init__(self, num_examples: int, rank: int = 0, world_size: int = 1, shuffle: bool = False,
                 seed: int = 0, drop_last: bool = True, batch_size: int = 1, mark_padding: bool = False):
        self.n = int(num_examples)
        self.rank, self.world = int(rank), int(world_size)
        self.shuffle, self.seed = shuffle, int(seed)
        self.drop_last = drop_last
        self.batch_size = int(batch_size)
        self.mark_padding = bool(mark_padding) and not drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def indices(self) -> List[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g).tolist()
        else:
            order = list(range(self.n))
        per_rank = self.n // self.world if self.drop_last else -(-self.n // self.world)
        if not self.drop_last:
            pad = order[: per_rank * self.world - self.n]
            order = order + ([-(i + 1) for i in pad] if self.mark_padding else pad)
        order = order[: per_rank * self.world]
        return order[self.rank::self.world]

    def batches(self) -> Iterator[List[int]]:
        idx = self.indices()
        nb = len(idx) // self.batch_size if self.drop_last else -(-len(idx) // self.batch_size)
        for b in range(nb):
            yield idx[b * self.batch_size:(b + 1) * self.batch_size]

    def num_batches(self) -> int:
        per_rank = len(self.indices())
        return per_rank // self.batch_size if self.drop_last else -(-per_rank // self.batch_size)
