"""Occupancy-grid culling (atmonr_amd.occupancy; beyond the reference).

* the compaction kernels keep exactly the samples whose cell is occupied, in order
  (torch restatement of the cell lookup on the same f32 ops), for ragged sizes, empty and
  full grids;
* with every cell occupied the culled pipeline equals the uniform one (outputs within
  1e-6, gradients within float-atomic noise);
* with a random grid, kept samples get bit-identical sigma / colour to the dense path and
  culled samples get exactly 0 (alpha 0 in the composite);
* training with the grid updating runs and lowers the loss.
"""

import pytest
import torch

import __graft_entry__ as ge

pytestmark = pytest.mark.gpu


def _torch_mask(x, occ, res, zmul):
    gx, gy, gz = res
    ix = torch.floor(x[:, 0] * gx).long().clamp(0, gx - 1)
    iy = torch.floor(x[:, 1] * gy).long().clamp(0, gy - 1)
    iz = torch.floor((x[:, 2] * zmul) * gz).long().clamp(0, gz - 1)
    return occ[(iz * gy + iy) * gx + ix] != 0


@pytest.mark.parametrize("M,fill", [(100003, 0.5), (1024, 0.3), (5, 0.5), (4096, 0.0),
                                    (3000, 1.0)])
def test_compact_matches_torch(dev, M, fill):
    from atmonr_amd.occupancy import OccupancyGrid

    g = torch.Generator().manual_seed(M)
    res = (16, 12, 8)
    grid = OccupancyGrid(res, alt_compress=8.0, warmup=0, max_fraction=1.0, device=dev)
    grid.set_occupancy(torch.rand(16 * 12 * 8, generator=g) < fill)
    x = torch.rand(M, 3, generator=g)
    x[:, 2] /= 8.0
    x[:7] = torch.tensor([0.0, 1.0, 1.0 / 8.0]).expand(7, 3) if M >= 7 else x[:7]
    x = x.to(dev)
    rows, kept = grid.compact(x)
    want = torch.nonzero(_torch_mask(x, grid.occ, res, 8.0)).flatten()
    assert torch.equal(rows.long(), want)
    assert torch.equal(kept, x[want])
    assert grid.last_fraction == pytest.approx(want.numel() / M)


@pytest.fixture(scope="module")
def scene(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    return SyntheticHARP2Dataset(n_views=8, img_size=32, device=dev, seed=0)


def _pipe(scene, dev, occ=None):
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    p = InstantNGPPipeline(ge._ingp_config(64), scene, dtype=torch.float16, fused=True,
                           seed=5, occupancy=occ)
    p.send_tensors_to(dev)
    return p


def test_all_occupied_equals_uniform(scene, dev):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.occupancy import OccupancyGrid

    a = _pipe(scene, dev)
    # max_fraction 1.0: the compacted (row-indirect) path runs although nothing is culled
    b = _pipe(scene, dev, OccupancyGrid(warmup=0, update_every=10 ** 9, max_fraction=1.0,
                                        device=dev))
    b.load_state_dict(a.state_dict())
    batch = next(iter(BatchLoader(scene, 512, seed=1)))
    u = torch.rand(512, 64, device=dev)
    ra, rb = a.forward(batch, u=u), b.forward(batch, u=u)
    assert b.occupancy.active and b.occupancy.last_fraction == 1.0
    for k in ("color_map_fine", "color_map_atmo", "color_map_surf", "sigma_fine"):
        assert (ra[k] - rb[k]).abs().max() <= 1e-6 * ra[k].abs().max() + 1e-12, k
    a.compute_loss(batch, ra).backward()
    b.compute_loss(batch, rb).backward()
    for m in ("pos_encoder", "pos_mlp", "dir_mlp"):
        ga, gb = getattr(a, m).params.grad, getattr(b, m).params.grad
        assert ((ga - gb).norm() / ga.norm()).item() <= 1e-4, m


def test_culled_samples_zero_kept_samples_exact(scene, dev):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.occupancy import OccupancyGrid

    a = _pipe(scene, dev)
    occ = OccupancyGrid((32, 32, 8), warmup=0, update_every=10 ** 9, device=dev)
    occ.set_occupancy(torch.rand(32 * 32 * 8, generator=torch.Generator().manual_seed(3)) < 0.4)
    b = _pipe(scene, dev, occ)
    b.load_state_dict(a.state_dict())
    batch = next(iter(BatchLoader(scene, 256, seed=2)))
    u = torch.rand(256, 64, device=dev)
    with torch.no_grad():
        ra, rb = a.forward(batch, u=u), b.forward(batch, u=u)
        from atmonr_amd.samplers import sample_and_preprocess

        _, _, coords = sample_and_preprocess(batch, 64, a._prep_ngp, u=u)
    keep = _torch_mask(coords.view(-1, 3), occ.occ, occ.res, occ.zmul).view(256, 64)[:, :-1]
    assert 0.05 < b.occupancy.last_fraction < 0.95
    for k in ("sigma_fine", "color_fine"):
        x, y = ra[k], rb[k]
        assert torch.equal(y[keep], x[keep]), k
        assert (y[~keep] == 0).all(), k


def test_training_with_grid_updates(scene, dev):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.occupancy import OccupancyGrid

    occ = OccupancyGrid((64, 64, 16), warmup=20, update_every=5, threshold=0.01, device=dev)
    p = _pipe(scene, dev, occ)
    opt = p.get_optimizer({"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15,
                           "weight_decay": 1e-2})
    losses, fracs = [], []
    for _ in range(4):
        for batch in BatchLoader(scene, 1024, seed=0):
            loss = p.compute_loss(batch, p.forward(batch))
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
            fracs.append(occ.last_fraction)
    assert occ.steps == len(losses) and occ.steps >= occ.warmup
    assert all(torch.isfinite(torch.tensor(losses)))
    assert sum(losses[-5:]) / 5 < 0.7 * sum(losses[:3]) / 3
    assert min(fracs) <= 1.0
