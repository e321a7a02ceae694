"""Data parallelism over rays (the one exchange step of the hot path).

The reference trains on one GPU only (scripts/train.py:94, trainer.py:33). Rays are
independent within a step and the loss is a batch mean, so W ranks that each process a
disjoint equal share of the global batch (atmonr_amd.batch_loader.BatchLoader with
rank / world_size) and average their gradients reproduce the single-process gradient of
the union batch. :class:`FlatGradBucket` makes every parameter's ``.grad`` a view into
one contiguous f32 buffer, so backward accumulates in place and a step needs exactly
one collective: ``all_reduce(AVG)`` of the whole buffer (RCCL over xGMI on MI355X;
gloo on CPU for the tests).
"""

from __future__ import annotations

from typing import Iterable

import torch
import torch.distributed as dist


class FlatGradBucket:
    def __init__(self, params: Iterable[torch.nn.Parameter], device=None):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = device if device is not None else self.params[0].device
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        self._known_zero = True
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero(self) -> None:
        """optimizer.zero_grad(set_to_none=False) for every bucketed param in one fill
        (skipped when the buffer is known to be zero already, see mark_zero)."""
        if not self._known_zero:
            self.flat.zero_()
        self._known_zero = False  # backward is about to accumulate into it

    def fuse_zero_into(self, optimizer) -> None:
        """Let a FusedAdam over (at least) every bucketed param zero the gradients in its
        update pass and mark this bucket zero after each step: the per-step fill goes."""
        optimizer.zero_grad_in_step = True
        optimizer.zeroed_buckets.append(self)

    def mark_zero(self) -> None:
        """The optimizer zeroed every gradient in its update pass (FusedAdam with
        zero_grad_in_step over all bucketed params): the next zero() needs no fill."""
        self._known_zero = True

    def all_reduce(self, group=None) -> None:
        """Average the gradient over the ranks of ``group`` (no-op when not distributed)."""
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=group)

    @property
    def numel(self) -> int:
        return self.flat.numel()
