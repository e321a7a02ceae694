"""BatchLoader — src/atmonr/batch_loader.py:9-52, device-resident and rank-sharded.

The reference builds each batch's index list on the CPU and copies it to the device
(batch_loader.py:30,47; survey §0 bug 6). Here the epoch permutation is drawn once on
the device and every batch is a slice of it. For data parallelism each of ``world_size``
ranks takes a disjoint, equal share of every global batch: rank r's k-th batch is
``perm[(k*W + r)*bs : (k*W + r + 1)*bs]`` of a permutation shared by all ranks
(same seed), so the union over ranks of one step is one global batch of W*bs rays.
"""

from __future__ import annotations

from collections.abc import Iterator

import torch


class BatchLoader:
    def __init__(self, dataset, batch_size: int, shuffle: bool = True, drop_last: bool = False,
                 rank: int = 0, world_size: int = 1, seed: int = 0):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.rank = rank
        self.world_size = world_size
        self.seed = seed
        self.epoch = 0
        self.n = len(dataset)
        self.device = getattr(dataset, "device", torch.device("cpu"))

    def _perm(self) -> torch.Tensor:
        if not self.shuffle:
            return torch.arange(self.n, device=self.device)
        g = torch.Generator(device=self.device if self.device.type == "cuda" else "cpu")
        g.manual_seed(self.seed * 1000003 + self.epoch)
        return torch.randperm(self.n, generator=g, device=self.device)

    def __len__(self) -> int:
        per_step = self.batch_size * self.world_size
        return self.n // per_step if self.drop_last else -(-self.n // per_step)

    def __iter__(self) -> Iterator[dict[str, torch.Tensor]]:
        perm = self._perm()
        self.epoch += 1
        bs, W = self.batch_size, self.world_size
        for k in range(len(self)):
            s = (k * W + self.rank) * bs
            idx = perm[s:s + bs]
            if idx.numel() == 0 or (self.drop_last and idx.numel() < bs):
                continue
            yield self.dataset.__getbatch__(idx)
