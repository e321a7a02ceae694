"""hipGraph capture of the train step (atmonr_amd.graph) and the device-step AdamW it needs
(anr_adam_step_multi_dev), on the GPU.

* anr_adam_step_multi_dev equals anr_adam_step_multi bit for bit over several steps,
  including a learning-rate change between steps (trainer.py:113-120's ExponentialLR
  writes group["lr"]; sync_hyper carries it to the device);
* a captured step replayed K times trains like K eager steps from the same start and the
  same batches: the two runs share every kernel, and differ only in the order in which
  the hash-grid backward's float atomics land, so losses and parameters agree to a
  tolerance, not bit for bit (tolerances below, measured ~1e-6 / ~1e-5);
* replays follow the loader's batches (the static index buffer is rewritten), and the
  device step count advances once per replay.
"""

import pytest
import torch

import __graft_entry__ as ge

pytestmark = pytest.mark.gpu

LOSS_RTOL = 2e-3     # per-step loss, captured vs eager (atomic order only)
PARAM_RTOL = 2e-3    # relative L2 of every module's parameters after the run


@pytest.fixture(scope="module")
def scene(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    return SyntheticHARP2Dataset(n_views=8, img_size=48, device=dev, seed=0)


def test_adam_dev_equals_host_step(dev):
    from atmonr_amd.optim import FusedAdam

    torch.manual_seed(0)
    shapes = [(1000,), (37, 5), (4096,)]
    init = [torch.randn(s, device=dev) for s in shapes]
    grads = [[torch.randn(s, device=dev) for s in shapes] for _ in range(5)]
    runs = []
    for capturable in (False, True):
        ps = [torch.nn.Parameter(x.clone()) for x in init]
        opt = FusedAdam([{"params": ps[:2], "weight_decay": 0.0},
                         {"params": ps[2:], "weight_decay": 1e-2}], lr=1e-2,
                        betas=(0.9, 0.99), eps=1e-15, capturable=capturable)
        for k in range(5):
            if k == 3:
                for g in opt.param_groups:
                    g["lr"] *= 0.33
            for p, g in zip(ps, grads[k]):
                p.grad = g.clone()
            opt.step()
        runs.append(([p.detach().clone() for p in ps],
                     [opt.state[p]["exp_avg_sq"].clone() for p in ps]))
        if capturable:
            assert opt.device_step() == 5
            sd = opt.state_dict()
            assert all(float(v["step"]) == 5.0 for v in sd["state"].values())
    for a, b in zip(runs[0][0] + runs[0][1], runs[1][0] + runs[1][1]):
        assert torch.equal(a, b)


def _job(scene, dev, graph):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.graph import GraphedTrainStep
    from atmonr_amd.parallel import FlatGradBucket
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    p = InstantNGPPipeline(ge._ingp_config(64), scene, dtype=torch.float16, fused=True, seed=3)
    p.send_tensors_to(dev)
    opt = p.get_optimizer({"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15,
                           "weight_decay": 1e-2})
    opt.capturable = graph
    bucket = FlatGradBucket([q for g in opt.param_groups for q in g["params"]], dev)
    bucket.fuse_zero_into(opt)
    bucket.enable_overlap()
    loader = BatchLoader(scene, 512, seed=2)
    g = GraphedTrainStep(p, scene, 512, opt, bucket) if graph else None
    return p, opt, bucket, loader, g


def _eager(p, opt, bucket, scene, idx):
    batch = scene.__getbatch__(idx)
    res = p.forward(batch)
    loss = p.compute_loss(batch, res)
    bucket.zero()
    loss.backward()
    bucket.all_reduce()
    opt.step()
    return loss


def test_graphed_step_matches_eager(scene, dev):
    K = 6
    losses = {}
    params = {}
    for graph in (False, True):
        torch.manual_seed(11)
        p, opt, bucket, loader, g = _job(scene, dev, graph)
        it = loader.index_batches()
        out = []
        for k in range(K):
            idx = next(it)
            if graph and k > 0:
                out.append(float(g(idx).item()))
            else:  # the first step runs eagerly (builds the lazy buffers), then capture
                out.append(float(_eager(p, opt, bucket, scene, idx).item()))
        torch.cuda.synchronize()
        losses[graph] = out
        params[graph] = {n: getattr(p, n).params.detach().clone() for n in p.module_names
                         if getattr(p, n).params.numel()}
        if graph:
            assert opt.device_step() == K
    for a, b in zip(losses[False], losses[True]):
        assert abs(a - b) <= LOSS_RTOL * abs(a), (losses[False], losses[True])
    assert len(set(losses[True])) == K  # the replays saw different batches
    for n, a in params[False].items():
        b = params[True][n]
        assert torch.linalg.norm(a - b) <= PARAM_RTOL * torch.linalg.norm(a), n


def test_graph_replay_after_load_state_dict(dev):
    """a checkpoint loaded into a capturable FusedAdam while a captured update
    is live. The loaded moments / step / lr are copied into the storage the graph points
    at, so replays continue from the loaded state: the update replayed for steps 3-4 after
    restoring the step-2 checkpoint (parameters + optimizer state) equals steps 3-4 of the
    uninterrupted run bit for bit, and no recapture is needed (same generation). (The
    whole train step is not compared this way: its stratified draws come from the device
    RNG, which a restore does not rewind.)"""
    import copy

    from atmonr_amd.optim import FusedAdam

    torch.manual_seed(3)
    shapes = [(4096,), (300, 7), (64,)]
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
    grads = [[torch.randn(s, device=dev) for s in shapes] for _ in range(5)]
    opt = FusedAdam([{"params": ps[:2], "weight_decay": 0.0},
                     {"params": ps[2:], "weight_decay": 1e-2}], lr=1e-2, betas=(0.9, 0.99),
                    eps=1e-15, capturable=True)
    for q, gr in zip(ps, grads[0]):
        q.grad = gr.clone()
    opt.step()  # eager: builds the device step / lr state
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        opt.step()

    def replay(k):
        for q, gr in zip(ps, grads[k]):
            q.grad.copy_(gr)
        opt.sync_hyper()
        graph.replay()

    for k in (1, 2):
        replay(k)
    torch.cuda.synchronize()
    ck_params = [q.detach().clone() for q in ps]
    ck_opt = copy.deepcopy(opt.state_dict())
    gen0 = opt.generation
    for k in (3, 4):
        replay(k)
    ref = [q.detach().clone() for q in ps]
    with torch.no_grad():
        for q, c in zip(ps, ck_params):
            q.copy_(c)
    opt.load_state_dict(ck_opt)
    assert opt.generation == gen0  # copied in place: the captured graph stays valid
    for k in (3, 4):
        replay(k)
    torch.cuda.synchronize()
    assert opt.device_step() == 5
    for a, q in zip(ref, ps):
        assert torch.equal(a, q.detach())
    # a lr written by a scheduler after the load still reaches the captured update
    for gp in opt.param_groups:
        gp["lr"] *= 0.5
    replay(4)
    torch.cuda.synchronize()
    assert all(torch.isfinite(q).all() for q in ps)
    # weight decay is captured by value, so a checkpoint carrying another
    # weight decay cannot be reloaded in place: the device state is dropped (recapture)
    ck_wd = copy.deepcopy(ck_opt)
    ck_wd["param_groups"][1]["weight_decay"] = 5e-2
    gen1 = opt.generation
    opt.load_state_dict(ck_wd)
    assert opt.generation > gen1


def test_adam_dev_rebuilds_when_grads_change(dev):
    """the device lr table follows launch order, so a parameter that loses its
    gradient (or gains one) must rebuild the capturable state, not shift every later
    tensor onto another tensor's lr. Capturable and plain FusedAdam stay bit-identical
    through such a change, and the rebuild bumps ``generation`` (a live graph would
    recapture)."""
    from atmonr_amd.optim import FusedAdam

    torch.manual_seed(1)
    shapes = [(100,), (300,), (50,)]
    init = [torch.randn(s, device=dev) for s in shapes]
    grads = [[torch.randn(s, device=dev) for s in shapes] for _ in range(4)]
    out = []
    gens = []
    for capturable in (False, True):
        ps = [torch.nn.Parameter(x.clone()) for x in init]
        opt = FusedAdam([{"params": ps[:1], "lr": 1e-2}, {"params": ps[1:], "lr": 3e-3}],
                        betas=(0.9, 0.99), eps=1e-15, weight_decay=0.0, capturable=capturable)
        for k in range(4):
            for j, (q, gr) in enumerate(zip(ps, grads[k])):
                # step 2: the first parameter has no gradient (skipped by both forms)
                q.grad = None if (k == 2 and j == 0) else gr.clone()
            opt.step()
            gens.append(opt.generation) if capturable else None
        out.append([q.detach().clone() for q in ps])
    for a, b in zip(*out):
        assert torch.equal(a, b)
    assert gens[2] > gens[1] and gens[3] > gens[2]  # rebuilt at the change and back
