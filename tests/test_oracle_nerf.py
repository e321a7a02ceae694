"""Pin the NeRF CPU-baseline restatement (oracle/ref_nerf.py) to the reference."""

import numpy as np
import torch

from oracle import ref_nerf
from tests.conftest import golden


def test_atmonerf_forward_matches_reference():
    g = golden("nerf.npz")
    net = ref_nerf.RefAtmoNeRF(76, 24, 4, 1, hidden=32).eval()
    sd = {k[len("nerf_w_"):]: torch.from_numpy(g[k]) for k in g.files if k.startswith("nerf_w_")}
    net.load_state_dict(sd)
    color, sigma = net(torch.from_numpy(g["nerf_x"]))
    np.testing.assert_allclose(color.detach().numpy(), g["nerf_color"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(sigma.detach().numpy(), g["nerf_sigma"], rtol=1e-6, atol=1e-7)


def test_sample_pdf_matches_reference():
    g = golden("sample_pdf.npz")
    t = {k: torch.from_numpy(g[k]) for k in g.files}
    pts, z = ref_nerf.sample_pdf(t["origin"], t["dir"], t["w"], t["zc"], 128, u=t["u"])
    assert torch.equal(z, t["z"])
    assert torch.equal(pts, t["pts"])


def test_preprocess_torch_matches_numpy_restatement():
    from oracle import ref_path

    g = golden("preprocess.npz")
    scale, lat_min, lat_range, lon_min, lon_range, h0, shift = g["std_meta"]
    pts = torch.from_numpy(g["std_pts"])
    out = ref_nerf.preprocess_torch(pts, float(scale), torch.from_numpy(g["std_offset"]),
                                    torch.tensor(lat_min, dtype=torch.float32),
                                    torch.tensor(lat_range, dtype=torch.float32),
                                    torch.tensor(lon_min, dtype=torch.float32),
                                    torch.tensor(lon_range, dtype=torch.float32), h0)
    assert np.abs(out.numpy() - g["std_coords"]).max() <= 2e-7
