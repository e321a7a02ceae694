"""Scene ingest: get_rays -> normalize_rays (wgs_84.py:223-339) against the
rays the reference itself produced for tests/golden/preprocess.npz (oracle/gen_golden.py),
bit for bit on CPU; horizontal <-> cartesian round trip."""

import numpy as np
import pytest
import torch

from tests.conftest import golden


@pytest.mark.parametrize("tag,lat0,lon0", [("std", 30.0, -60.0), ("dateline", -10.0, 179.9)])
def test_rays_match_reference_golden(tag, lat0, lon0):
    from atmonr_amd.geospatial import wgs_84

    g = golden("preprocess.npz")
    n = 24
    lat = (lat0 + (torch.arange(n, dtype=torch.float32) - n / 2)[:, None] * 0.0225
           + torch.zeros(1, 4)).float()
    lon = (lon0 + (torch.arange(n, dtype=torch.float32) - n / 2)[:, None] * 0.026
           + torch.zeros(1, 4)).float()
    lon = torch.where(lon > 180, lon - 360, lon)
    alt = torch.zeros_like(lat)
    thetav = torch.tensor([40.0, 10.0, 5.0, 30.0])[None].expand(n, 4).float()
    phiv = torch.tensor([0.0, 0.0, 180.0, 180.0])[None].expand(n, 4).float()
    o, d, ln = wgs_84.get_rays(lat, lon, alt, thetav, phiv, ray_origin_height=20000)
    o_n, scale, offset = wgs_84.normalize_rays(o, d, ln)
    assert torch.equal(o_n, torch.from_numpy(g[f"{tag}_ray_origin"]))
    assert torch.equal(d, torch.from_numpy(g[f"{tag}_ray_dir"]))
    assert torch.equal(ln / scale, torch.from_numpy(g[f"{tag}_ray_len"]))
    assert scale == float(g[f"{tag}_meta"][0])
    assert torch.equal(offset, torch.from_numpy(g[f"{tag}_offset"]))


def test_horizontal_cartesian_round_trip():
    from atmonr_amd.geospatial import wgs_84

    gen = torch.Generator().manual_seed(0)
    lat = (torch.rand(1000, generator=gen, dtype=torch.float64) - 0.5) * 160
    lon = (torch.rand(1000, generator=gen, dtype=torch.float64) - 0.5) * 358
    alt = torch.rand(1000, generator=gen, dtype=torch.float64) * 20000
    la, lo, al = wgs_84.cartesian_to_horizontal(*wgs_84.horizontal_to_cartesian(lat, lon, alt))
    # Bowring's one-step inverse (the reference's approximation): ~0.4 m in latitude at
    # 20 km, exact longitude
    assert np.abs((la - lat).numpy()).max() < 1e-5
    assert np.abs((lo - lon).numpy()).max() < 1e-9
    assert np.abs((al - alt).numpy()).max() < 1.0
