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
