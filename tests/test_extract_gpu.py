"""Extract path on the GPU (scripts/extract.py:180-211): the f64
preprocessor against the oracle in f64, and the batched extract loop against the same
kernels applied to the whole grid at once."""

import numpy as np
import pytest
import torch

import __graft_entry__ as ge
from oracle import ref_nerf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    return SyntheticHARP2Dataset(n_views=8, img_size=48, device=dev, seed=0)


def _oracle_coords_f64(pts64, pp, alt_compress=8.0):
    """harp2.py:372-386 in f64 on the CPU, then the INGP remap (instant_ngp.py:220-233)
    in f64, rounded to f32 where tcnn casts its input."""
    c = ref_nerf.preprocess_torch(pts64.cpu(), scale=float(pp.scale),
                                  offset=torch.tensor(pp.offset, dtype=torch.float64),
                                  lat_min=pp.lat_min, lat_range=pp.lat_range,
                                  lon_min=pp.lon_min, lon_range=pp.lon_range,
                                  h0=pp.ray_origin_height, shift_lon=pp.shift_lon)
    c = (c + 1) / 2
    c[..., 2] = c[..., 2] / alt_compress
    return c.float()


def test_preprocess_f64_matches_oracle(scene, dev):
    from atmonr_amd.samplers import preprocess_points

    pp = scene.get_point_preprocessor("horizontal")
    gen = torch.Generator().manual_seed(4)
    pts = (torch.rand(20000, 3, generator=gen, dtype=torch.float64) * 2 - 1) * torch.tensor(
        [1.1, 1.1, 0.4], dtype=torch.float64)
    out = preprocess_points(pts.to(dev), pp.params(ngp_remap=True, alt_compress=8.0))
    ref = _oracle_coords_f64(pts, pp)
    assert out.dtype == torch.float32 and out.shape == ref.shape
    # f64 libm (CPU) vs device f64 math: at most one f32 ulp after the final rounding
    err = (out.cpu() - ref).abs().max().item()
    assert err <= 1.2e-7, err
    with pytest.raises(Exception):
        preprocess_points(pts.to(dev).requires_grad_(True), pp.params())


def test_extract_volume_loop(scene, dev):
    from atmonr_amd.extract import GridExtractDataset, extract_volume
    from atmonr_amd.geospatial.wgs_84 import horizontal_to_cartesian
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    p = InstantNGPPipeline(ge._ingp_config(64), scene, seed=5)
    p.send_tensors_to(dev)
    p.eval()
    grid = GridExtractDataset(scene, alt_step=2000.0)
    A = grid.sample_alt.shape[0]
    assert A == 11 and len(grid) == 48 * 48 * A
    # grid points as harp2_extract.py:170-186 (CPU f64 vs device f64 math)
    lat = grid.lat.double().cpu()
    lon = grid.lon.double().cpu()
    alt = grid.sample_alt.double().cpu()[None, None].expand_as(lat)
    xyz = torch.stack(list(horizontal_to_cartesian(lat, lon, alt)), -1).view(-1, 3)
    assert (grid.xyz.cpu() - xyz).abs().max().item() < 1e-6
    sigma = extract_volume(p, scene, grid, batch_size=500)
    assert sigma.shape == (len(grid), 1) and bool((sigma >= 0).all())
    # the same kernels over the whole grid in one call
    pts = (grid.xyz - torch.as_tensor(scene.offset, dtype=torch.float64, device=dev)) / scene.scale
    direct = p.extract(pts).float() / scene.scale
    assert torch.equal(sigma, direct)
    # end to end against the oracle: f64 preprocessor coordinates -> restated tcnn hash grid
    # (f16 table, f16 features) -> pos MLP in f64 with the kernel's f16 roundings -> relu,
    # / scale (instant_ngp.py:208-247); tolerance 1e-2 of the largest value (f16 kernel)
    coords = _oracle_coords_f64(pts.cpu(), scene.get_point_preprocessor("horizontal"))
    from oracle import ref_tcnn

    table = p.pos_encoder.params.detach().half().double().cpu().numpy()
    enc = torch.from_numpy(ref_tcnn.hashgrid_fwd(coords.double().numpy(), table,
                                                 (3, 16, 16, 1.3819, 19)))
    pos_out = ref_tcnn.mlp_fwd(enc.half().double(), p.pos_mlp.params.detach().double().cpu(),
                               32, 16, p.pos_mlp.width, 1, half=True)
    ref_sigma = torch.clip(pos_out[:, :1], min=0) / scene.scale
    err = (sigma.double().cpu() - ref_sigma).abs().max().item()
    assert err <= 1e-2 * ref_sigma.abs().max().item() + 1e-12, err
    # dump round trip
    path = "/tmp/anr_extract_test.npz"
    grid.dump(path, sigma)
    d = np.load(path)
    assert d["extinction"].shape == (48, 48, A, 1) and d["sample_alt"].shape == (A,)


def test_extract_full_batch_spot_rows(scene, dev):
    """scripts/extract.py's batch shape: 32,768 columns x 81 altitudes (250 m steps to
    20 km) = 2,654,208 points in ONE pipeline.extract call (the bench's extract step).
    4,096 spot rows spread over the batch against the oracle (f64 preprocessor, restated
    tcnn hash grid, f16-rounded pos MLP), tolerance 1e-2 of the largest value (f16
    kernels); the batched loop equals one call over the whole grid."""
    from atmonr_amd.extract import GridExtractDataset, extract_volume
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_tcnn

    p = InstantNGPPipeline(ge._ingp_config(64), scene, seed=9)
    p.send_tensors_to(dev)
    p.eval()
    # a 256 x 128 lat/lon grid across the scene's footprint (the L1C grid stand-in)
    lat0, lon0 = scene.lat.min().item(), scene.lon.min().item()
    lat1, lon1 = scene.lat.max().item(), scene.lon.max().item()
    lat = torch.linspace(lat0, lat1, 256, device=dev)[:, None].expand(256, 128).contiguous()
    lon = torch.linspace(lon0, lon1, 128, device=dev)[None, :].expand(256, 128).contiguous()
    grid = GridExtractDataset(scene, alt_step=250.0, lat=lat, lon=lon)
    A = grid.sample_alt.shape[0]
    assert A == 81 and len(grid) == 32768 * 81
    sigma = extract_volume(p, scene, grid, batch_size=32768)
    halves = extract_volume(p, scene, grid, batch_size=16384)
    assert torch.equal(sigma, halves)
    # extract_volume hands the hash-grid walker the column length (81-point chunks); the
    # default chunking of a plain extract() call gives the same values
    off = torch.as_tensor(scene.offset, dtype=torch.float64, device=dev)
    plain = p.extract((grid.xyz - off) / scene.scale).float() / scene.scale
    assert torch.equal(sigma, plain)
    gen = torch.Generator().manual_seed(3)
    rows = torch.randint(0, len(grid), (4096,), generator=gen)
    pts = (grid.xyz[rows.to(dev)] - torch.as_tensor(scene.offset, dtype=torch.float64,
                                                     device=dev)) / scene.scale
    coords = _oracle_coords_f64(pts.cpu(), scene.get_point_preprocessor("horizontal"))
    table = p.pos_encoder.params.detach().half().double().cpu().numpy()
    enc = torch.from_numpy(ref_tcnn.hashgrid_fwd(coords.double().numpy(), table,
                                                 (3, 16, 16, 1.3819, 19)))
    pos_out = ref_tcnn.mlp_fwd(enc.half().double(), p.pos_mlp.params.detach().double().cpu(),
                               32, 16, p.pos_mlp.width, 1, half=True)
    ref_sigma = torch.clip(pos_out[:, :1], min=0) / scene.scale
    got = sigma[rows.to(dev)].double().cpu()
    err = (got - ref_sigma).abs().max().item()
    assert err <= 1e-2 * ref_sigma.abs().max().item() + 1e-12, err
    assert (ref_sigma > 0).any()
