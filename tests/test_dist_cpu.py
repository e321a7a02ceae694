"""World-size-2 data parallelism on CPU (gloo): rank-sharded batches are disjoint and
cover the global batch; the flat-bucket all-reduce averages gradients so that two ranks
reproduce the single-process gradient of the union batch."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Toy:
    def __init__(self, n):
        self.device = torch.device("cpu")
        self.x = torch.arange(n, dtype=torch.float32)

    def __len__(self):
        return self.x.shape[0]

    def __getbatch__(self, idx):
        return {"x": self.x[idx], "idx": idx}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import sys

    from tests.conftest import PKG

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.parallel import FlatGradBucket

    ds = _Toy(1000)
    idx = [b["idx"] for b in BatchLoader(ds, 64, rank=rank, world_size=world, seed=3)]
    # toy model: loss = mean over the rank's batch of (w * x - 1)^2
    w = torch.nn.Parameter(torch.tensor([0.5, -0.25]))
    bucket = FlatGradBucket([w], device=torch.device("cpu"))
    x = ds.x[idx[0]]
    loss = ((w[0] * x + w[1] - 1.0) ** 2).mean()
    bucket.zero()
    loss.backward()
    bucket.all_reduce()
    out[rank] = (torch.cat(idx).tolist(), w.grad.clone().tolist(), idx[0].tolist())
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_sharding_and_grad_average():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    seen0, g0, b0 = out[0]
    seen1, g1, b1 = out[1]
    # disjoint shards covering the epoch (1000 rays, 2 x 64 per step)
    assert not set(seen0) & set(seen1)
    assert len(set(seen0) | set(seen1)) == 1000
    # averaged gradient == single-process gradient of the union of the two first batches
    assert g0 == g1
    w = torch.nn.Parameter(torch.tensor([0.5, -0.25]))
    x = torch.tensor(b0 + b1, dtype=torch.float32)
    ((w[0] * x + w[1] - 1.0) ** 2).mean().backward()
    assert torch.allclose(torch.tensor(g0), w.grad, rtol=1e-6)


def _overlap_worker(rank, world, port, out):
    import sys

    from tests.conftest import PKG

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from atmonr_amd import _lib
    from atmonr_amd.parallel import FlatGradBucket

    class Direct(torch.autograd.Function):
        """y = x * p, accumulating dL/dp into p.grad itself (as the HIP modules do)."""

        @staticmethod
        def forward(ctx, x, p):
            ctx.save_for_backward(x, p)
            return x * p

        @staticmethod
        def backward(ctx, g):
            x, p = ctx.saved_tensors
            p.grad += (g * x).sum(0)
            order.append(("done", p._tag))
            _lib.grad_done(p)
            order.append(("issued", sum(w is not None for w in bucket._works)))
            return g * p, None

    order = []
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.full((n,), 0.1 * (i + 1))) for i, n in
          enumerate([4096, 3, 5, 2048])]
    for i, p in enumerate(ps):
        p._tag = i
    bucket = FlatGradBucket(ps, device=torch.device("cpu"))
    bucket.enable_overlap(min_chunk_bytes=4 * 1024)  # chunks: [p0], [p1, p2, p3]
    grads, local = [], []
    for step in range(2):
        x = torch.randn(8, 4096, generator=torch.Generator().manual_seed(10 * step + rank))
        # p0 feeds everything (its gradient is final last); p1..p3 act on the output
        _lib.grad_use(ps[0])
        h = Direct.apply(x, ps[0])
        _lib.grad_use(ps[3])
        a = Direct.apply(h[:, :2048], ps[3])
        _lib.grad_use(ps[1])
        b = Direct.apply(h[:, :3], ps[1])
        _lib.grad_use(ps[2])
        c = Direct.apply(h[:, :5], ps[2])
        _lib.grad_use(ps[2])  # p2 used twice: final only after both backward uses
        c2 = Direct.apply(h[:, 5:10], ps[2])
        loss = (a ** 2).mean() + b.sum() + (c * c2).sum()
        bucket.zero()
        loss.backward()
        issued_before = sum(w is not None for w in bucket._works)
        bucket.all_reduce()
        grads.append([p.grad.clone() for p in ps])
        # this rank's own gradient, plain autograd
        q = [p.detach().clone().requires_grad_(True) for p in ps]
        hq = x * q[0]
        ((hq[:, :2048] * q[3]) ** 2).mean().backward(retain_graph=True)
        ((hq[:, :3] * q[1]).sum() + ((hq[:, :5] * q[2]) * (hq[:, 5:10] * q[2])).sum()).backward()
        local.append([t.grad.clone() for t in q])
        if step == 0:
            out[f"order{rank}"] = list(order)
            out[f"early{rank}"] = (issued_before, bucket.early_issued)
        for p in ps:
            p.grad.zero_()
    out[rank] = [[g.tolist() for g in gs] for gs in grads]
    out[f"local{rank}"] = [[g.tolist() for g in gs] for gs in local]
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_overlapped_bucket_matches_plain_all_reduce():
    """enable_overlap: each chunk is all-reduced during the backward as soon as its
    gradients are final (not while a param still owes a backward use), the chunk of the
    first-used param last; the averaged gradients equal the ranks' own gradients
    averaged."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_overlap_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        issued_before, early = out[f"early{r}"]
        assert issued_before == 2 and early == 2  # both chunks issued inside backward
        order = out[f"order{r}"]
        # the chunk [p1, p2, p3] is issued right after its last completion, not before
        dones = [i for i, e in enumerate(order) if e[0] == "done"]
        first_issue = next(i for i, e in enumerate(order) if e[0] == "issued" and e[1] == 1)
        finals = [order[i][1] for i in dones if i < first_issue]
        assert sorted(set(finals)) == [1, 2, 3] and finals.count(2) == 2
        assert order[-2] == ("done", 0) and order[-1] == ("issued", 2)  # [p0] last
    g0, g1 = out[0], out[1]
    assert g0 == g1
    for step in range(2):
        for k in range(4):
            want = (torch.tensor(out["local0"][step][k]) + torch.tensor(out["local1"][step][k])) / 2
            assert torch.allclose(torch.tensor(g0[step][k]), want, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("n,bs,W", [(1000, 100, 8), (1000, 450, 2), (23587960, 1024, 8),
                                    (1000, 64, 2), (7, 4, 8), (1024, 128, 8)])
def test_loader_equal_steps_and_shares(n, bs, W):
    """Every rank yields len(loader) batches, all ranks' batches of a step have one size,
    shards are disjoint, and only the rem % W tail rays are dropped (ranks
    yielding different batch counts mismatch the DP collectives)."""
    from atmonr_amd.batch_loader import BatchLoader

    loaders = [BatchLoader(_Len(n), bs, rank=r, world_size=W, seed=0)
               for r in range(W)]
    sl = [ld.slices() for ld in loaders]
    L = len(loaders[0])
    assert all(len(ld) == L and len(s) == L for ld, s in zip(loaders, sl))
    covered = 0
    for k in range(L):
        sizes = {e - s for s, e in (x[k] for x in sl)}
        assert len(sizes) == 1 and sizes.pop() > 0
        covered += sum(e - s for s, e in (x[k] for x in sl))
    starts = sorted(x for s in sl for x in s)
    assert all(a[1] <= b[0] for a, b in zip(starts, starts[1:]))  # disjoint
    full = n // (bs * W)
    rem = n - full * bs * W
    assert covered == full * bs * W + (rem // W) * W


class _Len:
    device = torch.device("cpu")

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def test_loader_iterates_tail_shares():
    from atmonr_amd.batch_loader import BatchLoader

    ds = _Toy(1000)
    got = [[b["idx"] for b in BatchLoader(ds, 100, rank=r, world_size=8, seed=5)]
           for r in range(8)]
    assert [len(g) for g in got] == [2] * 8
    assert {g[1].numel() for g in got} == {25}
    allidx = torch.cat([t for g in got for t in g])
    assert allidx.unique().numel() == 1000


def _reference_adamw(segments, step, betas, eps, decoupled):
    """The K10 kernel's arithmetic (adam.hip) in torch, for the CPU tests of ShardedAdam."""
    import math

    b1, b2 = betas
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    for s in segments:
        p, g = s.param, s.grad
        if s.weight_decay:
            p.mul_(1 - s.lr * s.weight_decay)
        s.exp_avg.lerp_(g, 1 - b1)
        s.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (s.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(s.exp_avg, denom, value=-s.lr / bc1)
        if s.shadow is not None:
            s.shadow.copy_(p)


def _sharded_worker(rank, world, port, gather, out):
    import sys

    from tests.conftest import PKG

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from atmonr_amd.parallel import FlatGradBucket, ShardSegment, ShardedAdam

    sizes = [37, 5, 1000, 3, 129]  # shards straddle parameter boundaries

    def make():
        g = torch.Generator().manual_seed(1)
        return [torch.nn.Parameter(torch.randn(n, generator=g) * 0.1) for n in sizes]

    def groups(ps):  # as InstantNGPPipeline.get_optimizer: two groups, wd on the second
        return [{"params": ps[:2], "weight_decay": 0.0, "lr": 1e-2},
                {"params": ps[2:], "weight_decay": 1e-2, "lr": 3e-3}]

    def loss_of(ws, step):
        x = torch.randn(16, sum(sizes), generator=torch.Generator().manual_seed(100 * step + rank))
        w = torch.cat([t.reshape(-1) for t in ws])
        return ((x * w).sum(1) ** 2).mean() + (w ** 3).sum()

    betas, eps = (0.9, 0.99), 1e-15
    # (a) all-reduce of the flat bucket + the replicated update over whole parameters
    pa = make()
    ba = FlatGradBucket(pa, device=torch.device("cpu"))
    hp = {id(p): (g["lr"], g["weight_decay"]) for g in groups(pa) for p in g["params"]}
    st = {id(p): (torch.zeros_like(p), torch.zeros_like(p)) for p in pa}
    # (b) ShardedAdam
    pb = make()
    bb = FlatGradBucket(pb, device=torch.device("cpu"), pad_to=world)
    opt = ShardedAdam(bb, groups(pb), betas=betas, eps=eps, gather=gather,
                      update=_reference_adamw)
    for step in range(1, 5):
        # forward on what the kernels would read: the f16 copy in gather="f16" mode
        fa = [p.detach().half().float().requires_grad_(False) if gather == "f16" else p
              for p in pa]
        if gather == "f16":
            for p, f in zip(pa, fa):
                f.requires_grad_(True)
        ba.zero()
        la = loss_of(fa, step)
        la.backward()
        if gather == "f16":
            for p, f in zip(pa, fa):
                p.grad.copy_(f.grad)
        ba.all_reduce()
        with torch.no_grad():
            segs = [ShardSegment(param=p.data.view(-1), grad=p.grad.view(-1),
                                 exp_avg=st[id(p)][0].view(-1), exp_avg_sq=st[id(p)][1].view(-1),
                                 shadow=None, lr=hp[id(p)][0], weight_decay=hp[id(p)][1])
                    for p in pa]
            _reference_adamw(segs, step, betas, eps, True)
        fb = [p._anr_shadow.float().requires_grad_(True) if gather == "f16" else p for p in pb]
        bb.zero()
        lb = loss_of(fb, step)
        lb.backward()
        if gather == "f16":
            for p, f in zip(pb, fb):
                p.grad.copy_(f.grad)
        opt.step()
        if gather == "f16":  # the gathered f16 copies equal the replicated path's f16 params
            for p, q in zip(pa, pb):
                assert torch.allclose(q._anr_shadow.float(), p.detach().half().float(),
                                      rtol=2e-3, atol=1e-6)
    opt.consolidate()
    out[rank] = ([p.detach().clone() for p in pa], [p.detach().clone() for p in pb],
                 opt.state_numel(), sum(sizes))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,gather", [(2, "f32"), (2, "f16"), (8, "f32"), (8, "f16")])
def test_sharded_adam_matches_all_reduce_path(world, gather):
    """ShardedAdam (reduce-scatter, AdamW on 1/W of the parameters, all-gather) against the
    all-reduce + replicated AdamW path after 4 steps, at world sizes 2 and 8 (gloo):
    parameters equal on every rank (to the f32 summation-order noise of the two
    collectives), optimizer state 2n/W per rank."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sharded_worker, args=(world, _free_port(), gather, out), nprocs=world, join=True)
    ref = out[0][0]
    for r in range(world):
        pa, pb, state, n = out[r]
        for a, b, c in zip(pa, pb, ref):
            assert torch.equal(a, c)  # the replicated path: identical on every rank
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (r, (a - b).abs().max())
        assert state == 2 * (-(-n // world))


def _sharded_sched_worker(rank, world, port, out):
    import sys

    from tests.conftest import PKG

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torch.optim.lr_scheduler import ExponentialLR

    from atmonr_amd.parallel import FlatGradBucket, ShardedAdam

    sizes = [37, 5, 1000, 3, 129]

    def make():
        g = torch.Generator().manual_seed(1)
        return [torch.nn.Parameter(torch.randn(n, generator=g) * 0.1) for n in sizes]

    def build(ps):
        b = FlatGradBucket(ps, device=torch.device("cpu"), pad_to=world)
        # the second group leaves weight_decay to the optimizer's default (AdamW's 1e-2)
        opt = ShardedAdam(b, [{"params": ps[:2], "weight_decay": 0.0, "lr": 1e-2},
                              {"params": ps[2:], "lr": 3e-3}], betas=(0.9, 0.99), eps=1e-15,
                          gather="f32", update=_reference_adamw)
        return b, opt

    def step(ps, b, opt, k):
        x = torch.randn(16, sum(sizes), generator=torch.Generator().manual_seed(100 * k + rank))
        b.zero()
        w = torch.cat([t.reshape(-1) for t in ps])
        (((x * w).sum(1) ** 2).mean() + (w ** 3).sum()).backward()
        opt.step()

    # (a) ShardedAdam under ExponentialLR (trainer.py:113-120), 5 steps straight through
    pa = make()
    ba, oa = build(pa)
    assert oa.param_groups[1]["weight_decay"] == 1e-2
    sa = ExponentialLR(oa, gamma=0.5)
    for k in range(5):
        step(pa, ba, oa, k)
        sa.step()
    # (b) 3 steps, checkpoint (torch AdamW layout), a fresh optimizer loads it, 2 more
    pb = make()
    bb, ob = build(pb)
    sb = ExponentialLR(ob, gamma=0.5)
    for k in range(3):
        step(pb, bb, ob, k)
        sb.step()
    sd = ob.state_dict()
    assert set(sd["state"][2]) == {"step", "exp_avg", "exp_avg_sq"}
    assert sd["state"][2]["exp_avg"].shape == (1000,) and float(sd["state"][0]["step"]) == 3
    pc = [torch.nn.Parameter(p.detach().clone()) for p in pb]
    bc, oc = build(pc)
    oc.load_state_dict(sd)
    assert oc.param_groups[1]["lr"] == 3e-3 * 0.125 and oc.steps == 3
    for k in range(3, 5):
        step(pc, bc, oc, k)
        for g in oc.param_groups:
            g["lr"] *= 0.5
    # a torch.optim.AdamW loads the same checkpoint
    t = torch.optim.AdamW([{"params": make()[:2]}, {"params": make()[2:]}])
    t.load_state_dict(sd)
    out[rank] = ([p.detach().clone() for p in pa], [p.detach().clone() for p in pc],
                 [g["lr"] for g in oa.param_groups])
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_adam_scheduler_and_checkpoint():
    """ShardedAdam is a torch Optimizer with live param groups: ExponentialLR's lr reaches
    its updates; state_dict() (torch AdamW layout, moments all-gathered) loaded into a
    fresh ShardedAdam continues bit-identically to an uninterrupted run, and loads into
    torch.optim.AdamW (gloo, world size 2)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sharded_sched_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        pa, pc, lrs = out[r]
        assert lrs == [1e-2 * 0.5 ** 5, 3e-3 * 0.5 ** 5]
        for a, c in zip(pa, pc):
            assert torch.equal(a, c)


def _f16_exchange_worker(rank, world, port, out):
    import sys

    from tests.conftest import PKG

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from atmonr_amd.parallel import FlatGradBucket, ShardedAdam

    sizes = [37, 5, 1000, 3, 129]
    res = {}
    for exchange in ("f32", "f16"):
        g0 = torch.Generator().manual_seed(1)
        ps = [torch.nn.Parameter(torch.randn(n, generator=g0) * 0.1) for n in sizes]
        b = FlatGradBucket(ps, device=torch.device("cpu"), pad_to=world)
        opt = ShardedAdam(b, [{"params": ps[:2], "weight_decay": 0.0, "lr": 1e-2},
                              {"params": ps[2:], "weight_decay": 1e-2, "lr": 3e-3}],
                          betas=(0.9, 0.99), eps=1e-15, gather="f32",
                          update=_reference_adamw, exchange=exchange)
        for step in range(4):
            b.zero()
            gg = torch.Generator().manual_seed(1000 * step + rank)
            with torch.no_grad():
                for p in ps:  # tinycudann-style per-rank gradients: f16 numbers, many tiny
                    v = torch.randn(p.shape, generator=gg) * torch.exp(
                        torch.randn(p.shape, generator=gg) * 4) * 1e-4
                    p.grad.copy_(v.half().float())
            opt.step()
        res[exchange] = [p.detach().clone() for p in ps]
        if exchange == "f16":  # a gradient that is not an f16 number is refused
            with torch.no_grad():
                ps[0].grad.fill_(0.1)
            opt.steps = 0  # the check runs on the first step ...
            try:
                opt.step()
                res["refused"] = False
            except ValueError:
                res["refused"] = True
            opt.check_every = 8  # ... and every check_every steps after it
            opt.steps = 16
            try:
                opt.step()
                res["refused_later"] = False
            except ValueError:
                res["refused_later"] = True
            with torch.no_grad():  # a NaN is not reported as a non-f16 value
                ps[0].grad.copy_(ps[0].grad.half().float())
                ps[0].grad[0] = float("nan")
            opt.steps = 0
            try:
                opt.step()
                res["nan_passes"] = True
            except ValueError:
                res["nan_passes"] = False
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 8])
def test_sharded_adam_f16_exchange(world):
    """ShardedAdam(exchange="f16"): the gradient slices go through one f16 all-to-all and
    are summed in f32 on their owner (half the bytes of the f32 reduce-scatter). With
    f16-valued gradients (the reference numerics' tinycudann gradients) the parameters
    after 4 steps equal the f32 reduce-scatter path's to f32 summation order, at world
    sizes 2 and 8 (gloo); non-f16 gradients are refused."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_f16_exchange_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        res = out[r]
        assert res["refused"] and res["refused_later"] and res["nan_passes"]
        for a, b in zip(res["f32"], res["f16"]):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), (r, (a - b).abs().max())
        for a, b in zip(out[0]["f16"], res["f16"]):
            assert torch.equal(a, b)  # every replica identical
