"""Reference-produced state and device ingest on the GPU.

* f4: the AtmoNeRF state dict the REFERENCE produced (tests/golden/nerf.npz, written by
  oracle/gen_golden.py from models/nerf.py) loads into NeRFPipeline's coarse network
  through the pipeline's nested {"coarse", "fine"} state dict (pipelines/nerf.py:242-273)
  and reproduces the reference's forward on the golden inputs (f32 library GEMMs: 1e-5
  of the largest value); the pipeline's state dict hands the same keys back.
* f2: get_rays -> normalize_rays (wgs_84.py:223-339) on the device, against the rays the
  reference produced for tests/golden/preprocess.npz. f64 libm on the GPU differs from
  glibc in the last ulp, which can move the reference's f32-rounded ECEF surface point
  by one f32 ulp (0.5 m); the bar is 1 m / scale for origins and lengths and 4 f32 ulps
  for directions (the CPU test, tests/test_scene_cpu.py, is bit-exact).
"""

import pytest
import torch

from tests.conftest import golden

pytestmark = pytest.mark.gpu


def test_reference_nerf_state_dict_loads_and_reproduces_forward(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.nerf import NeRFPipeline

    g = golden("nerf.npz")
    sd_ref = {k[len("nerf_w_"):]: torch.from_numpy(g[k]) for k in g.files
              if k.startswith("nerf_w_")}
    ds = SyntheticHARP2Dataset(n_views=4, img_size=8, device=dev, seed=0)
    cfg = {"type": "NeRF", "include_height": False, "point_preprocessor": "horizontal",
           "num_bands": 4, "ray_origin_height": 20000, "sampler": {"N_c": 64, "N_f": 128},
           "encoder": {"L_x": [14, 14, 10], "L_d": 4}, "mlp_hidden_dim": 32}
    p = NeRFPipeline(cfg, ds)
    p.send_tensors_to(dev)
    full = p.state_dict()
    assert set(full) == {"coarse", "fine"} and set(full["coarse"]) == set(sd_ref)
    p.load_state_dict({"coarse": sd_ref, "fine": full["fine"]})
    p.eval()
    with torch.no_grad():
        color, sigma = p.nerf["coarse"](torch.from_numpy(g["nerf_x"]).to(dev))
    rc, rs = torch.from_numpy(g["nerf_color"]), torch.from_numpy(g["nerf_sigma"])
    assert (color.cpu() - rc).abs().max().item() <= 1e-5 * rc.abs().max().item() + 1e-7
    assert (sigma.cpu() - rs).abs().max().item() <= 1e-5 * rs.abs().max().item() + 1e-7
    back = p.state_dict()["coarse"]
    for k, v in sd_ref.items():
        assert torch.equal(back[k].cpu(), v), k


@pytest.mark.parametrize("tag,lat0,lon0", [("std", 30.0, -60.0), ("dateline", -10.0, 179.9)])
def test_device_rays_match_reference_golden(dev, tag, lat0, lon0):
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
    o, d, ln = wgs_84.get_rays(lat.to(dev), lon.to(dev), alt.to(dev), thetav.to(dev),
                               phiv.to(dev), ray_origin_height=20000)
    assert o.is_cuda and d.is_cuda
    o_n, scale, offset = wgs_84.normalize_rays(o, d, ln)
    ro, rd = torch.from_numpy(g[f"{tag}_ray_origin"]), torch.from_numpy(g[f"{tag}_ray_dir"])
    rl = torch.from_numpy(g[f"{tag}_ray_len"])
    # origins and lengths come from surface points the reference rounds from f64 ECEF
    # metres (|x| ~ 6.4e6 m) to f32, whose ulp is 0.5 m: a last-ulp difference between the
    # device's and glibc's f64 sin / cos moves a point by 0.5 m, i.e. 0.5 / scale in the
    # normalized frame. Bar: 2 such ulps (1 m / scale); directions (unit vectors through
    # the rotation matmuls): 4 f32 ulps of 1.
    tol_m = 1.0 / float(g[f"{tag}_meta"][0])
    eps = torch.finfo(torch.float32).eps
    for name, got, ref, tol in (("origin", o_n.cpu(), ro, tol_m), ("dir", d.cpu(), rd, 4 * eps),
                                ("len", (ln / scale).cpu(), rl, tol_m)):
        err = (got - ref).abs().max().item()
        assert err <= tol, (name, err, tol)
    assert abs(float(scale) - float(g[f"{tag}_meta"][0])) <= 1e-9 * float(g[f"{tag}_meta"][0])
    # offset in metres, from the f32 extrema of the rays (1 m = 2 f32 ulps of ECEF)
    assert (offset.cpu().double() - torch.from_numpy(g[f"{tag}_offset"]).double()).abs().max() < 1.0
