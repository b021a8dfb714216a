"""Rank-sharded sampling (DistributedSampler equivalent, no torch.distributed dependency)."""
from __future__ import annotations

from typing import Iterator

import torch
from torch.utils.data import Sampler


class ShardedSampler(Sampler[int]):
    """Every rank sees a disjoint ``1/world`` slice of a (seeded, per-epoch) permutation.
    ``drop_last=False`` pads by wrapping so all ranks take the same number of steps
    (required: every rank must issue the same collective sequence)."""

    def __init__(self, n: int, rank: int = 0, world_size: int = 1, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        self.n, self.rank, self.world = n, rank, world_size
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last:
            self.per_rank = n // world_size
        else:
            self.per_rank = (n + world_size - 1) // world_size

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __iter__(self) -> Iterator[int]:
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        total = self.per_rank * self.world
        if len(idx) < total:
            idx = (idx * ((total // max(1, len(idx))) + 1))[:total]
        idx = idx[:total]
        return iter(idx[self.rank:total:self.world])

    def __len__(self) -> int:
        return self.per_rank
