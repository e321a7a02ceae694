"""Data parallelism over rays (the one exchange step of the hot path).

The reference trains on one GPU only (scripts/train.py:94, trainer.py:33). Rays are
independent within a step and the loss is a batch mean, so W ranks that each process a
disjoint equal share of the global batch (atmonr_amd.batch_loader.BatchLoader with
rank / world_size) and average their gradients reproduce the single-process gradient of
the union batch. :class:`FlatGradBucket` makes every parameter's ``.grad`` a view into
one contiguous f32 buffer, so backward accumulates in place and a step needs exactly
one collective: ``all_reduce(AVG)`` of the whole buffer (RCCL over xGMI on MI355X;
gloo on CPU for the tests).

Overlap (``enable_overlap``): the buffer is cut into chunks along parameter boundaries and
a chunk's all-reduce is issued (async, stream-ordered behind the kernel that finished its
last gradient) as soon as every parameter in it is done for the step, so it runs while the
rest of the backward computes. The Instant-NGP step produces the surface network's and
the MLPs' gradients before the 3-D hash grid's (the last backward kernel): their
all-reduce hides behind the hash-grid backward. Modules report uses and completions
(``_lib.grad_use`` before a forward that will write a bucketed gradient directly,
``_lib.grad_done`` after the backward kernel that wrote it); a parameter is done when its
completions have caught up with its uses. ``all_reduce()`` issues whatever is left and
waits for everything. Not for gradient accumulation over several backward passes per
step (a chunk could be reduced before the later passes add to it).
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

    # ------------------------------------------------------------------ overlap
    def enable_overlap(self, min_chunk_bytes: int = 4 << 20, group=None) -> None:
        """Issue each chunk's all-reduce as soon as its gradients are final (see module
        doc). Chunks: consecutive parameters merged until ``min_chunk_bytes``."""
        self._group = group
        self._chunks = []  # (start, end, [param index])
        start, idx = 0, []
        off = 0
        for i, p in enumerate(self.params):
            idx.append(i)
            off += p.numel()
            if 4 * (off - start) >= min_chunk_bytes or i == len(self.params) - 1:
                self._chunks.append((start, off, idx))
                start, idx = off, []
        self._chunk_of = {}
        for c, (_, _, ids) in enumerate(self._chunks):
            for i in ids:
                self._chunk_of[id(self.params[i])] = c
        for p in self.params:
            p._anr_bucket = self
        self._pending = {id(p): 0 for p in self.params}
        self._used = set()  # params registered through grad_use this step
        self._works = [None] * len(self._chunks)
        self._done_ev = {}  # chunk -> events on the streams its gradients were finished on
        self.early_issued = 0  # chunks issued before all_reduce() in the last step
        self._early = 0

    @property
    def overlap(self) -> bool:
        return hasattr(self, "_chunks")

    def _distributed(self, group=None) -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1

    def grad_use(self, p) -> None:
        if self.overlap and id(p) in self._pending:
            self._pending[id(p)] += 1
            self._used.add(id(p))

    def grad_done(self, p) -> None:
        if not self.overlap or id(p) not in self._pending:
            return
        self._pending[id(p)] -= 1
        c = self._chunk_of[id(p)]
        if self.flat.is_cuda and self._distributed(self._group):
            # the stream this gradient was finished on (the surface branch runs on a side
            # stream): the chunk's all-reduce waits for every such stream, not only the
            # one current when the chunk's last gradient completes
            ev = torch.cuda.Event()
            ev.record()
            self._done_ev.setdefault(c, []).append(ev)
        # a chunk is ready only when every param in it reported its uses this step and
        # all of them completed: a param whose gradient autograd accumulates on its own
        # (never reported) keeps its chunk for all_reduce(), after the whole backward
        if self._works[c] is None and all(
                id(self.params[i]) in self._used and self._pending[id(self.params[i])] <= 0
                for i in self._chunks[c][2]):
            self._issue(c)
            self._early += 1

    def _issue(self, c) -> None:
        s, e, _ = self._chunks[c]
        if self._distributed(self._group):
            if self.flat.is_cuda:
                cur = torch.cuda.current_stream(self.flat.device)
                for ev in self._done_ev.pop(c, ()):
                    cur.wait_event(ev)
            self._works[c] = dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.AVG,
                                             group=self._group, async_op=True)
        else:
            self._works[c] = True

    def all_reduce(self, group=None) -> None:
        """Average the gradient over the ranks of ``group`` (no-op when not distributed).
        With overlap: issue the chunks not yet issued, then wait for all of them (stream
        waits for RCCL, so the optimizer kernels queue behind the collectives)."""
        if self.overlap:
            for c in range(len(self._chunks)):
                if self._works[c] is None:
                    self._issue(c)
            for w in self._works:
                if w is not True and w is not None:
                    w.wait()
            self.early_issued = self._early
            self._works = [None] * len(self._chunks)
            self._done_ev = {}
            self._pending = {k: 0 for k in self._pending}
            self._used = set()
            self._early = 0
            return
        if self._distributed(group):
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=group)

    def broadcast_params(self, src: int = 0, group=None) -> None:
        """Make every rank start from rank ``src``'s parameters (replicas whose init draws
        from an unseeded RNG would otherwise train different weights on one averaged
        gradient). Cached f16 compute copies are invalidated."""
        if not self._distributed(group):
            return
        with torch.no_grad():
            for p in self.params:
                dist.broadcast(p.data, src=src, group=group)
                if hasattr(p, "_anr_shadow_ver"):
                    p._anr_shadow_ver = None

    @property
    def numel(self) -> int:
        return self.flat.numel()
