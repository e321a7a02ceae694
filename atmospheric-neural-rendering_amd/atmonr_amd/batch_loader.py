"""BatchLoader — src/atmonr/batch_loader.py:9-52, device-resident and rank-sharded.

The reference builds each batch's index list on the CPU and copies it to the device
(batch_loader.py:30,47; survey §0 bug 6). Here the epoch permutation is drawn once on
the device and every batch is a slice of it. For data parallelism each of ``world_size``
ranks takes a disjoint, equal share of every global batch: rank r's k-th batch is
``perm[(k*W + r)*bs : (k*W + r + 1)*bs]`` of a permutation shared by all ranks
(same seed), so the union over ranks of one step is one global batch of W*bs rays.

Epoch tail (the last global step holds ``rem < W*bs`` rays): every rank takes an equal
``rem // W`` share of it and the ``rem % W`` leftover rays are dropped, so all ranks run
the same number of steps (their collectives stay matched) and the rank-averaged gradient
is the gradient of the union batch. If ``rem < W`` the tail step is dropped on every
rank. At ``world_size == 1`` this is the reference's ``drop_last=False`` behaviour.
"""

from __future__ import annotations

from collections.abc import Iterator

import torch


class BatchLoader:
    def __init__(self, dataset, batch_size: int, shuffle: bool = True, drop_last: bool = False,
                 rank: int = 0, world_size: int = 1, seed: int = 0):
        if not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} outside world size {world_size}")
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.rank = rank
        self.world_size = world_size
        self.seed = seed
        self.epoch = 0  # the next epoch's permutation index (Trainer.load restores it)
        self.n = len(dataset)
        self.device = getattr(dataset, "device", torch.device("cpu"))

    def _perm(self) -> torch.Tensor:
        if not self.shuffle:
            return torch.arange(self.n, device=self.device)
        g = torch.Generator(device=self.device if self.device.type == "cuda" else "cpu")
        g.manual_seed(self.seed * 1000003 + self.epoch)
        return torch.randperm(self.n, generator=g, device=self.device)

    def _tail_share(self) -> int:
        """Rays per rank in the last, partial global step (0: no such step)."""
        if self.drop_last:
            return 0
        rem = self.n % (self.batch_size * self.world_size)
        return rem // self.world_size

    def __len__(self) -> int:
        full = self.n // (self.batch_size * self.world_size)
        return full + (1 if self._tail_share() > 0 else 0)

    def slices(self) -> list[tuple[int, int]]:
        """(start, end) into the epoch permutation of this rank's batches, in order."""
        bs, W, r = self.batch_size, self.world_size, self.rank
        full = self.n // (bs * W)
        out = [((k * W + r) * bs, (k * W + r + 1) * bs) for k in range(full)]
        q = self._tail_share()
        if q > 0:
            base = full * W * bs
            out.append((base + r * q, base + (r + 1) * q))
        return out

    def index_batches(self) -> Iterator[torch.Tensor]:
        """The ray indices of this rank's batches of the next epoch (device int64 slices of
        the permutation): what __iter__ gathers, for callers that gather themselves (a
        captured step reads its rows from a static index buffer, atmonr_amd.graph)."""
        perm = self._perm()
        self.epoch += 1
        for s, e in self.slices():
            yield perm[s:e]

    def __iter__(self) -> Iterator[dict[str, torch.Tensor]]:
        perm = self._perm()
        self.epoch += 1
        for s, e in self.slices():
            yield self.dataset.__getbatch__(perm[s:e])
