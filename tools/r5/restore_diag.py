"""Diagnostic (r05): restore a step-2 checkpoint and replay steps 3-4, graph and eager."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]
import torch  # noqa: E402

from tests.test_graph_gpu import _job, _eager  # noqa: E402
from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset  # noqa: E402

dev = torch.device("cuda:0")
scene = SyntheticHARP2Dataset(n_views=8, img_size=48, device=dev, seed=0)
for graph in (False, True):
    torch.manual_seed(11)
    p, opt, bucket, loader, g = _job(scene, dev, graph)
    it = loader.index_batches()
    idx = [next(it) for _ in range(5)]
    run = (lambda i: g(i)) if graph else (lambda i: _eager(p, opt, bucket, scene, i))
    _eager(p, opt, bucket, scene, idx[0])
    for k in (1, 2):
        run(idx[k])
    torch.cuda.synchronize()
    names = [n for n in p.module_names if getattr(p, n).params.numel()]
    ck = {n: getattr(p, n).params.detach().clone() for n in names}
    ck_opt = copy.deepcopy(opt.state_dict())
    res = {}
    for rep in range(3):
        if rep:
            with torch.no_grad():
                for n in names:
                    getattr(p, n).params.copy_(ck[n])
            opt.load_state_dict(ck_opt)
        ls = [float(run(idx[k]).item()) for k in (3, 4)]
        res[rep] = (ls, {n: getattr(p, n).params.detach().clone() for n in names})
    for rep in (1, 2):
        d = {n: (torch.linalg.norm(res[rep][1][n] - res[0][1][n]) /
                 torch.linalg.norm(res[0][1][n])).item() for n in names}
        print("graph" if graph else "eager", "rep", rep, res[0][0], res[rep][0], d, flush=True)
