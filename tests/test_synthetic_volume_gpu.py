"""The synthetic scene's volume-truth mode (datasets/synthetic.py, radiance_model="volume"):
each ray's radiance is the reference's render_with_surface (graphics_utils.py:6-77,
restated in oracle/ref_path.py and pinned there by tests/golden/render.npz) of a known
extinction field, so trained or extracted extinction can be scored against ground truth
(SURVEY §8 d).
"""

import numpy as np
import pytest
import torch

from oracle import ref_path

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vol(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    return SyntheticHARP2Dataset(n_views=4, img_size=24, device=dev, seed=3,
                                 radiance_model="volume", truth_samples=96)


def test_volume_radiance_is_reference_render_of_truth(vol):
    """Ray radiance == oracle render_with_surface of (z km, cloud colour, truth sigma,
    surface colour) on the same bin midpoints and preprocessed sample positions (1e-6)."""
    from atmonr_amd.samplers import preprocess_points

    n = 96
    # the rays the truth field changes most (through a blob), and three spread ones
    surf_all = vol._surface(vol.lat.reshape(-1)[vol.ray_filter].double(),
                            vol.lon.reshape(-1)[vol.ray_filter].double(), vol.ray_irgb_idx) * 100.0
    moved = (vol.ray_rad.double() - surf_all).abs() / surf_all
    rows = torch.cat([moved.topk(4).indices,
                      torch.linspace(0, len(vol) - 1, 3).long().to(moved.device)])
    t = (torch.arange(n, dtype=torch.float64, device=rows.device) + 0.5) / n
    z = t[None] * vol.ray_len_norm[rows].double()[:, None]
    pts = vol.ray_origin_norm[rows].double()[:, None] + vol.ray_dir[rows].double()[:, None] * z[..., None]
    c = preprocess_points(pts.float(), vol.get_point_preprocessor("horizontal").params()).double()
    lat, lon, alt = vol._coords_to_horizontal(c)
    sig = vol.extinction_truth(lat, lon, alt)
    band = vol.ray_irgb_idx[rows]
    cloud = torch.tensor(vol.CLOUD_COLOR, dtype=torch.float64)[band.cpu()] * 100.0
    surf = vol._surface(vol.lat.reshape(-1)[vol.ray_filter][rows].double(),
                        vol.lon.reshape(-1)[vol.ray_filter][rows].double(), band).cpu() * 100.0
    zk = (z * (float(vol.scale) / 1000.0)).cpu()
    col = cloud[:, None, None].expand(-1, n, 1).contiguous()
    rad, alpha, _, atmo, surf_term = ref_path.render_with_surface(
        zk, col, sig.cpu()[..., None], surf[:, None])
    got = vol.ray_rad[rows].double().cpu()
    np.testing.assert_allclose(got.numpy(), rad[:, 0].numpy(), rtol=1e-6)
    # the truth field is visible: some rays see optical depth well above zero
    assert float((alpha.sum(dim=1)).max()) > 0.05


def test_volume_mode_shapes_and_truth_scoring(vol):
    assert vol.radiance_model == "volume"
    assert torch.isfinite(vol.ray_rad).all() and float(vol.ray_rad.min()) > 0
    assert vol.max_i == pytest.approx(float(vol.ray_rad.max()))
    # target cube and ray radiance agree (the cube is built from ray_rad)
    cube = vol.target_image()
    assert cube.shape == (4, 24, 24)
    # scoring the truth against itself: r = 1, unit scale, zero error; a scaled copy
    # is recovered up to its scale
    lat = vol.lat[:, 0].double()
    lon = vol.lon[:, 0].double()
    alt = torch.full_like(lat, 3000.0)
    truth = vol.extinction_truth(lat, lon, alt)
    s = vol.score_extinction(truth, lat, lon, alt)
    assert s["pearson_r"] == pytest.approx(1.0, abs=1e-12)
    assert s["rel_l2_after_scale"] < 1e-12
    s2 = vol.score_extinction(truth * 250.0, lat, lon, alt)
    assert s2["scale"] == pytest.approx(1 / 250.0, rel=1e-12)


def test_parallax_mode_unchanged(dev):
    """The benchmark scene (parallax model) is untouched by the volume option."""
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    a = SyntheticHARP2Dataset(n_views=4, img_size=16, device=dev, seed=1)
    b = SyntheticHARP2Dataset(n_views=4, img_size=16, device=dev, seed=1,
                              radiance_model="parallax")
    assert torch.equal(a.ray_rad, b.ray_rad)
    c = SyntheticHARP2Dataset(n_views=4, img_size=16, device=dev, seed=1,
                              radiance_model="volume", truth_samples=32)
    assert not torch.equal(a.ray_rad, c.ray_rad)
    assert torch.equal(a.ray_dir, c.ray_dir)


def test_extract_grid_geometry_matches_truth_coordinates(vol):
    """The scoring geometry: the extract path's query points (lat, lon, alt -> WGS-84 xyz
    -> normalized scene -> horizontal preprocessor, scripts/extract.py:203-207) land on
    the same (lat, lon, alt) that :meth:`extinction_truth` is evaluated at for ray samples
    (the preprocessor's normalisation inverted), so a trained field is compared with the
    truth at the right places."""
    from atmonr_amd.extract import GridExtractDataset
    from atmonr_amd.samplers import preprocess_points

    grid = GridExtractDataset(vol, alt_step=2500.0)
    off = torch.as_tensor(vol.offset, dtype=torch.float64, device=grid.xyz.device)
    pts = (grid.xyz - off) / vol.scale
    c = preprocess_points(pts, vol.get_point_preprocessor("horizontal").params()).double()
    lat, lon, alt = vol._coords_to_horizontal(c)
    want_alt = grid.sample_alt[None, None].expand_as(grid.lat).reshape(-1).double()
    inside = (c.abs() < 0.999).all(dim=1)  # the clip at the domain faces moves points
    assert int(inside.sum()) > 0.5 * inside.numel()
    assert float((lat - grid.lat.reshape(-1).double())[inside].abs().max()) < 1e-4
    assert float((lon - grid.lon.reshape(-1).double())[inside].abs().max()) < 1e-4
    assert float((alt - want_alt)[inside].abs().max()) < 5.0
