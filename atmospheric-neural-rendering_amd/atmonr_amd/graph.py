"""hipGraph capture of the Instant-NGP train step (trainer.py:99-105 as one graph launch).

The reference's step (forward -> compute_loss -> zero_grad -> backward -> optimizer.step,
src/atmonr/trainer.py:99-105) costs ~50 kernel launches here. At the per-rank shape of
8-GPU strong scaling (1,024 rays x 1,024 samples) the host needs longer to issue them
through Python and autograd (0.9 ms) than the GPU needs to run them, so the step is
host-bound. :class:`GraphedTrainStep` captures the whole step once with
``torch.cuda.graph`` (hipStreamBeginCapture / hipGraphInstantiate underneath; the libanr
entry points launch on torch's current stream, so they are captured like torch's own
kernels) and replays it with ONE hipGraphLaunch per step.

What changes between replays lives in device memory the graph reads:

* the batch's ray indices: ``static_idx`` (a slice of the loader's device-resident epoch
  permutation is copied into it before each replay; the gather kernel reads it);
* the uniform draws: torch's Philox generator, registered with the graph by torch (each
  replay advances its offset, as eager ``torch.rand`` would);
* the AdamW step count and learning rates: FusedAdam(capturable=True) keeps them on the
  device (anr_adam_step_multi_dev); ``sync_hyper`` writes a changed lr before a replay.

Everything else a step allocates comes from the graph's private memory pool and is
reused by every replay. Collectives are not captured: with a data-parallel bucket whose
all-reduce or ShardedAdam runs after backward, pass ``optimizer_in_graph=False`` and the
replay is followed by the eager exchange + update (3 launches).
"""

from __future__ import annotations

from typing import Callable

import torch

from . import _lib


class GraphedTrainStep:
    """One captured train step of ``pipe`` on ``dataset`` rows ``static_idx``.

    ``optimizer_in_graph``: the (capturable FusedAdam) update is part of the graph;
    otherwise ``after`` (e.g. ``lambda: (bucket.all_reduce(), opt.step())``) runs eagerly
    after each replay. ``bucket``: the FlatGradBucket holding every gradient; the graph
    zeroes it at its start unless the in-graph optimizer zeroes it in its update pass.
    """

    def __init__(self, pipe, dataset, batch_size: int, optimizer, bucket=None,
                 optimizer_in_graph: bool = True, after: Callable[[], None] | None = None):
        if optimizer_in_graph and not getattr(optimizer, "capturable", False):
            raise _lib.ANRError("GraphedTrainStep: an in-graph optimizer must be "
                                "FusedAdam(capturable=True)")
        if bucket is not None and bucket.overlap and bucket._distributed():
            raise _lib.ANRError("GraphedTrainStep: collectives are not captured; disable the "
                                "bucket's overlapped all-reduce and run it in `after`")
        self.pipe, self.dataset, self.optimizer, self.bucket = pipe, dataset, optimizer, bucket
        self.optimizer_in_graph = optimizer_in_graph
        self.after = after
        dev = dataset.device
        self.device = dev
        self.static_idx = torch.zeros(batch_size, dtype=torch.int64, device=dev)
        self.graph = None
        self.loss = None

    def _body(self):
        opt, bucket = self.optimizer, self.bucket
        # a FusedAdam that zeroes the bucket in its update pass (in the graph or in `after`)
        # leaves it zero for the next replay; otherwise the graph zeroes it itself
        fused_zero = (getattr(opt, "zero_grad_in_step", False) and bucket is not None
                      and any(b is bucket for b in getattr(opt, "zeroed_buckets", ())))
        if bucket is not None and not fused_zero:
            bucket.flat.zero_()  # part of the graph: every replay starts from zero
        batch = self.dataset.__getbatch__(self.static_idx)
        res = self.pipe.forward(batch)
        loss = self.pipe.compute_loss(batch, res)
        loss.backward()
        if bucket is not None and bucket.overlap and not bucket._distributed():
            bucket.all_reduce()  # one process: resets the chunk bookkeeping, no collective
        if self.optimizer_in_graph:
            opt.step()
        return loss

    def capture(self, idx: torch.Tensor, timer=None) -> None:
        """Capture the step (after at least one eager step of the same shape, so every
        lazily built buffer and the optimizer's device state exist). Nothing runs during
        the capture: the first replay is the first step. ``timer``: a
        _lib.KernelTimer(external=True) whose events become nodes of the graph."""
        if self.bucket is not None:
            self.bucket._known_zero = False  # the graph decides its own zeroing
        self.static_idx.copy_(idx)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        saved = _lib._timer
        _lib._timer = timer  # no timing events inside the capture unless asked
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.loss = self._body()
        finally:
            _lib._timer = saved
        self.graph = g
        self._opt_generation = getattr(self.optimizer, "generation", 0)
        if self.bucket is not None and self.optimizer_in_graph:
            # the captured AdamW zeroes the bucket in its pass (or the graph's own fill
            # does): eager code after a replay sees zero gradients
            self.bucket._known_zero = True

    def _refresh_compute_copies(self) -> None:
        """A parameter torch modified since the capture (a checkpoint's load_state_dict,
        ``copy_``) has a stale f16 compute copy: the replay reads the copy, and only the
        eager forward would notice the version change. Rewrite such copies in place (same
        storage, so the graph's pointers stay valid) before replaying."""
        for group in self.optimizer.param_groups:
            for p in group["params"]:
                sh = getattr(p, "_anr_shadow", None)
                if sh is not None and getattr(p, "_anr_shadow_ver", None) != p._version:
                    _lib.compute_copy(p, sh.dtype)

    def __call__(self, idx: torch.Tensor) -> torch.Tensor:
        """One step on rows ``idx`` (device int64, the captured batch size)."""
        if (self.graph is not None and self.optimizer_in_graph
                and getattr(self.optimizer, "generation", 0) != self._opt_generation):
            # the optimizer replaced tensors the graph points at (e.g. a load_state_dict
            # that could not copy in place): rebuild its device state eagerly, recapture
            self.graph = None
            self.optimizer._prepare()
        if self.graph is None:
            self.capture(idx)
        elif idx.data_ptr() != self.static_idx.data_ptr():
            self.static_idx.copy_(idx)
        if self.optimizer_in_graph:
            self.optimizer.sync_hyper()
        self._refresh_compute_copies()
        self.graph.replay()
        if self.after is not None:
            self.after()
        return self.loss
