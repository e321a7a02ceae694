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
    def __init__(self, params: Iterable[torch.nn.Parameter], device=None, pad_to: int = 1):
        """``pad_to``: round the buffer up to a multiple (ShardedAdam's rank count; the
        tail past the last parameter stays zero)."""
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        self.n_params = n
        n = -(-n // pad_to) * pad_to
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


class ShardSegment:
    """The part of one parameter inside this rank's shard: views into the flat buffers
    (``param``, ``grad``, ``exp_avg``, ``exp_avg_sq``, ``shadow`` f16 or None) and its
    group's ``lr`` / ``weight_decay`` (refreshed from the live param group every step)."""

    __slots__ = ("param", "grad", "exp_avg", "exp_avg_sq", "shadow", "lr", "weight_decay",
                 "group")

    def __init__(self, **kw):
        self.group = None
        for k, v in kw.items():
            setattr(self, k, v)


def hip_adam_update(segments, step: int, betas, eps: float, decoupled: bool) -> None:
    """Adam(W) over the shard's segments in one anr_adam_step_multi launch (the K10
    kernel FusedAdam uses)."""
    import ctypes

    from . import _lib

    if not segments:
        return
    ts = [_lib.AdamTensor(_lib.ptr(s.param), _lib.ptr(s.grad), _lib.ptr(s.exp_avg),
                          _lib.ptr(s.exp_avg_sq), _lib.ptr(s.shadow), s.param.numel(),
                          float(s.lr), float(s.weight_decay), int(step)) for s in segments]
    arr = (_lib.AdamTensor * len(ts))(*ts)
    dev = segments[0].param.device
    _lib.call("anr_adam_step_multi", ctypes.addressof(arr), len(ts), float(betas[0]),
              float(betas[1]), float(eps), int(decoupled), 0, _lib.stream(dev), tag="adam")


class ShardedAdam(torch.optim.Optimizer):
    """Optimizer sharded over the data-parallel ranks (ZeRO stage 1), the alternative to
    FlatGradBucket.all_reduce + a replicated FusedAdam:

    1. ``reduce_scatter(AVG)`` of the flat gradient bucket: rank r receives the averaged
       gradient of its slice [r*S, (r+1)*S) of the flat parameter vector;
    2. Adam(W) on that slice only (state for 1/W of the parameters; per-parameter lr and
       weight decay of its param group, as the replicated optimizer);
    3. ``all_gather`` of the updated slice: ``gather="f16"`` gathers the f16 compute copy
       the forward kernels read (half the bytes of f32; the f32 masters outside the slice
       are then stale until :meth:`consolidate`, which :meth:`state_dict` calls),
       ``gather="f32"`` gathers the f32 parameters (every replica stays complete; the f16
       copies refresh from them on the next forward).

    A torch Optimizer over the given param groups: ``param_groups`` stay live, so a
    scheduler writing ``group["lr"]`` (trainer.py:113-120's ExponentialLR) reaches the
    next step; ``state_dict()`` / ``load_state_dict()`` use torch.optim.AdamW's format
    (per-parameter ``step`` / ``exp_avg`` / ``exp_avg_sq``, the moments all-gathered), so
    checkpoints interchange with FusedAdam's and torch's at any rank count. A group
    without ``weight_decay`` gets FusedAdam's default (AdamW's 1e-2 when decoupled, Adam's
    0 otherwise).

    Bytes per step: reduce-scatter 4n + all-gather 2n (f16) against the all-reduce's 8n
    (a ring all-reduce is a reduce-scatter plus an all-gather of f32), and the AdamW pass
    over n / W elements. ``exchange="f16"`` (r05) sends the gradient slices as f16 through
    one all-to-all and sums the W received slices in f32 on the owner -- 2n + 2n bytes,
    exact when every gradient value is an f16 number, as under the reference numerics
    (tinycudann's f16 parameter gradients, quantised per rank before the exchange); a
    gradient that is not f16-exact is refused (``check_f16``: on the first step and every
    ``check_every`` steps). Parameters become views into one flat f32 buffer (padded to a
    multiple of W). ``update(segments, step, betas, eps, decoupled)`` applies the update
    (default: the HIP multi-tensor kernel; tests inject a reference)."""

    def __init__(self, bucket: FlatGradBucket, param_groups: list, betas=(0.9, 0.999),
                 eps: float = 1e-8, decoupled: bool = True, gather: str = "f16", group=None,
                 update=hip_adam_update, lr: float = 1e-3, weight_decay: float | None = None,
                 exchange: str = "f32", check_f16: bool = True, check_every: int = 256):
        if gather not in ("f16", "f32"):
            raise ValueError("gather: 'f16' or 'f32'")
        if exchange not in ("f16", "f32"):
            raise ValueError("exchange: 'f16' or 'f32'")
        self.exchange, self.check_f16 = exchange, check_f16
        self.check_every = max(1, int(check_every))
        if weight_decay is None:  # FusedAdam's default: torch.optim.AdamW's 1e-2, Adam's 0
            weight_decay = 1e-2 if decoupled else 0.0
        super().__init__(param_groups, dict(lr=lr, betas=tuple(betas), eps=eps,
                                            weight_decay=weight_decay))
        self.bucket, self.group, self.gather = bucket, group, gather
        self.betas, self.eps, self.decoupled = tuple(betas), float(eps), decoupled
        self.update = update
        self.world = dist.get_world_size(group) if bucket._distributed(group) else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        n_pad = bucket.flat.numel()
        if n_pad % self.world:
            raise ValueError("FlatGradBucket must be padded to a multiple of the rank count "
                             "(FlatGradBucket(..., pad_to=world_size))")
        self.S = n_pad // self.world
        dev = bucket.flat.device
        owner = {id(p): g for g in self.param_groups for p in g["params"]}
        # flat f32 parameters: every parameter becomes a view into it
        self.flat_param = torch.zeros(n_pad, device=dev, dtype=torch.float32)
        off = 0
        self._spans = []  # (param, offset)
        with torch.no_grad():
            for p in bucket.params:
                if id(p) not in owner:
                    raise ValueError("every bucketed parameter must be in a param group")
                n = p.numel()
                self.flat_param[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat_param[off:off + n].view_as(p)
                self._spans.append((p, off))
                off += n
        lo, hi = self.rank * self.S, (self.rank + 1) * self.S
        self.grad_shard = torch.zeros(self.S, device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros(self.S, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(self.S, device=dev, dtype=torch.float32)
        self.flat_shadow = self.shadow_shard = None
        if gather == "f16":
            self.flat_shadow = self.flat_param.to(torch.float16)
            self.shadow_shard = torch.zeros(self.S, device=dev, dtype=torch.float16)
            for p, o in self._spans:
                p._anr_shadow = self.flat_shadow[o:o + p.numel()].view_as(p)
                p._anr_shadow_ver = p._version
        self.segments = []
        for p, o in self._spans:
            a, b = max(o, lo), min(o + p.numel(), hi)
            if a >= b:
                continue
            g = owner[id(p)]
            self.segments.append(ShardSegment(
                param=self.flat_param[a:b], grad=self.grad_shard[a - lo:b - lo],
                exp_avg=self.exp_avg[a - lo:b - lo], exp_avg_sq=self.exp_avg_sq[a - lo:b - lo],
                shadow=None if self.shadow_shard is None else self.shadow_shard[a - lo:b - lo],
                lr=float(g["lr"]), weight_decay=float(g["weight_decay"]), group=g))
        self.steps = 0
        self.masters_current = True

    @torch.no_grad()
    def step(self, closure=None):
        """Reduce-scatter, update this rank's slice, all-gather (call after backward, in
        place of bucket.all_reduce() + optimizer.step())."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lo = self.rank * self.S
        if self.world > 1 and self.exchange == "f16":
            half = self.bucket.flat.to(torch.float16)
            # checked on the first step and every check_every steps after it (a guard
            # against pairing it with f32 gradients, e.g. a module added to the bucket
            # without the end-of-backward quantisation); NaN entries are not compared (a
            # non-finite gradient is the loss scaler's business, not a layout error)
            if self.check_f16 and self.steps % self.check_every == 0:
                flat = self.bucket.flat
                same = (half.float() == flat) | torch.isnan(flat)
                if not bool(same.all()):
                    raise ValueError(
                        "ShardedAdam(exchange='f16'): the gradient holds values that are not "
                        "f16 numbers (quantise them first, or exchange in f32)")
            recv = torch.empty_like(half)
            # slice r of every rank's gradient lands on rank r: recv[j * S:(j + 1) * S] is
            # rank j's contribution, summed here in f32 in rank order
            dist.all_to_all_single(recv, half, group=self.group)
            torch.sum(recv.view(self.world, self.S).float(), 0, out=self.grad_shard)
            self.grad_shard.div_(self.world)
        elif self.world > 1:
            dist.reduce_scatter_tensor(self.grad_shard, self.bucket.flat, op=dist.ReduceOp.AVG,
                                       group=self.group)
        else:
            self.grad_shard.copy_(self.bucket.flat[lo:lo + self.S])
        self.steps += 1
        for sg in self.segments:  # the live group's hyper-parameters (schedulers write them)
            sg.lr = float(sg.group["lr"])
            sg.weight_decay = float(sg.group["weight_decay"])
        self.update(self.segments, self.steps, self.betas, self.eps, self.decoupled)
        mine = self.flat_param[lo:lo + self.S]
        if self.gather == "f16":
            if self.world > 1:
                dist.all_gather_into_tensor(self.flat_shadow, self.shadow_shard, group=self.group)
            else:
                self.flat_shadow.copy_(self.shadow_shard)
            self.masters_current = self.world == 1
            for p, _ in self._spans:
                p._anr_shadow_ver = p._version  # the gathered f16 copy is current
                p._anr_master_stale = not self.masters_current
        else:
            if self.world > 1:
                dist.all_gather_into_tensor(self.flat_param, mine.clone(), group=self.group)
            for p, _ in self._spans:
                if hasattr(p, "_anr_shadow_ver"):
                    p._anr_shadow_ver = None  # refresh the f16 copy from the gathered f32
        self.bucket._known_zero = False
        return loss

    def zero_grad(self, set_to_none: bool = False) -> None:
        """The gradients are views into the bucket: zero it (never set to None)."""
        self.bucket.zero()

    @torch.no_grad()
    def consolidate(self) -> None:
        """All-gather the f32 master slices so every replica holds every parameter (before
        a checkpoint or an evaluation on the f32 weights; f16 gather only)."""
        if self.masters_current:
            return
        lo = self.rank * self.S
        dist.all_gather_into_tensor(self.flat_param, self.flat_param[lo:lo + self.S].clone(),
                                    group=self.group)
        self.masters_current = True
        for p, _ in self._spans:
            p._anr_master_stale = False
            if hasattr(p, "_anr_shadow_ver"):
                p._anr_shadow_ver = p._version

    def _gathered(self, shard: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return shard.clone()
        full = torch.empty(self.S * self.world, device=shard.device, dtype=shard.dtype)
        dist.all_gather_into_tensor(full, shard.contiguous(), group=self.group)
        return full

    def state_dict(self) -> dict:
        """torch.optim.AdamW's layout for every parameter (a collective: call on every
        rank). Consolidates the f32 masters first."""
        self.consolidate()
        m, v = self._gathered(self.exp_avg), self._gathered(self.exp_avg_sq)
        span = {id(p): o for p, o in self._spans}
        index, groups, state = {}, [], {}
        for g in self.param_groups:
            ids = []
            for p in g["params"]:
                k = index.setdefault(id(p), len(index))
                ids.append(k)
                o, n = span[id(p)], p.numel()
                state[k] = {"step": torch.tensor(float(self.steps)),
                            "exp_avg": m[o:o + n].view_as(p).clone(),
                            "exp_avg_sq": v[o:o + n].view_as(p).clone()}
            groups.append({**{k: v for k, v in g.items() if k != "params"}, "params": ids})
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, state_dict: dict) -> None:
        """Load a torch.optim.AdamW / FusedAdam / ShardedAdam state dict (same parameter
        order): this rank keeps its slice of the moments; group hyper-parameters are
        copied into the live groups."""
        groups = state_dict["param_groups"]
        if len(groups) != len(self.param_groups):
            raise ValueError("state dict has a different number of param groups")
        span = {id(p): o for p, o in self._spans}
        lo = self.rank * self.S
        steps = set()
        for g, sg in zip(self.param_groups, groups):
            if len(g["params"]) != len(sg["params"]):
                raise ValueError("param group sizes differ from the state dict's")
            for k, v in sg.items():
                if k != "params":
                    g[k] = v
            for p, key in zip(g["params"], sg["params"]):
                st = state_dict["state"].get(key)
                if not st:
                    continue
                steps.add(int(float(st["step"])))
                o, n = span[id(p)], p.numel()
                a, b = max(o, lo), min(o + n, lo + self.S)
                if a < b:
                    self.exp_avg[a - lo:b - lo].copy_(st["exp_avg"].reshape(-1)[a - o:b - o])
                    self.exp_avg_sq[a - lo:b - lo].copy_(st["exp_avg_sq"].reshape(-1)[a - o:b - o])
        if len(steps) > 1:
            raise ValueError("ShardedAdam keeps one step count: parameters at different steps")
        self.steps = steps.pop() if steps else 0

    def state_numel(self) -> int:
        return 2 * self.S
