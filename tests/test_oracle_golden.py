"""Pin the oracle to the reference: oracle restatement vs golden vectors produced by the
reference's own code (oracle/gen_golden.py). CPU only."""

import numpy as np
import pytest
import torch

from oracle import ref_path
from tests.conftest import golden


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_sampler_bit_exact(tag):
    g = golden("sampler.npz")
    o, d, ln, u = (torch.from_numpy(g[f"{tag}_{k}"]) for k in ("origin", "dir", "len", "u"))
    N = u.shape[1]
    pts, z = ref_path.sample_uniform_bins(o, d, ln, u, N)
    assert torch.equal(z, torch.from_numpy(g[f"{tag}_z"]))
    assert torch.equal(pts, torch.from_numpy(g[f"{tag}_pts"]))
    pts, z = ref_path.sample_uniform_bins(o, d, ln, None, N)
    assert torch.equal(z, torch.from_numpy(g[f"{tag}_z_mid"]))
    assert torch.equal(pts, torch.from_numpy(g[f"{tag}_pts_mid"]))


def test_reference_sampler_bounds_fixture():
    """The reference's only test (tests/test_samplers.py:9-28) on the oracle."""
    og = torch.from_numpy(np.mgrid[-1:1.01:0.1, -1:1.01:0.1, -1:1.01:0.1].astype(np.float32))
    og = og.reshape(3, -1).T
    torch.manual_seed(6558903984)
    u = torch.rand(og.shape[0], 64)
    pts, z = ref_path.sample_uniform_bins(og, -og, torch.zeros(og.shape[0]) + 2, u, 64)
    assert (pts >= -1).all() and (pts <= 1).all()
    assert (z >= 0).all() and (z <= 2).all()


@pytest.mark.parametrize("tag", ["std", "dateline"])
def test_preprocessor(tag):
    g = golden("preprocess.npz")
    meta = g[f"{tag}_meta"]
    scale, lat_min, lat_range, lon_min, lon_range, h0, shift = meta
    out = ref_path.preprocess_horizontal(g[f"{tag}_pts"], scale, g[f"{tag}_offset"], lat_min,
                                         lat_range, lon_min, lon_range, h0, bool(shift))
    ref = g[f"{tag}_coords"]
    # fp64 transcendental libraries differ by ulps; after the f32 cast nearly all agree
    assert np.abs(out - ref).max() <= 2e-7
    assert (out == ref).mean() > 0.99


def test_render_f32():
    g = golden("render.npz")
    for tag in ("f32", "f32long", "f32multi"):
        z, c, s, cs = (torch.from_numpy(g[f"{tag}_{k}"]) for k in ("z", "color", "sigma", "cs"))
        zz = z.clone().requires_grad_(True)
        cc, ss, css = (t.clone().requires_grad_(True) for t in (c, s, cs))
        cm, alpha, w, atmo, surf = ref_path.render_with_surface(zz, cc, ss, css)
        for name, t in [("cm", cm), ("alpha", alpha), ("w", w), ("atmo", atmo), ("surf", surf)]:
            np.testing.assert_allclose(t.detach().numpy(), g[f"{tag}_{name}"], rtol=1e-6, atol=1e-7)
        loss = ((cm * torch.from_numpy(g[f"{tag}_gcm"])).sum()
                + (atmo * torch.from_numpy(g[f"{tag}_gatmo"])).sum()
                + (surf * torch.from_numpy(g[f"{tag}_gsurf"])).sum()
                + (w * torch.from_numpy(g[f"{tag}_gw"])).sum())
        loss.backward()
        for name, t in [("dz", zz), ("dcolor", cc), ("dsigma", ss), ("dcs", css)]:
            np.testing.assert_allclose(t.grad.numpy(), g[f"{tag}_{name}"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["dark", "hdr", "l1", "l1_plus_hdr", "mse", "mse_plus_hdr"])
def test_losses(name):
    g = golden("losses.npz")
    p = torch.from_numpy(g["pred"]).requires_grad_(True)
    val = ref_path.LOSSES[name](p, torch.from_numpy(g["gt"]), float(g["max_i"]))
    val.backward()
    np.testing.assert_allclose(val.item(), g[f"{name}_val"], rtol=1e-6)
    np.testing.assert_allclose(p.grad.numpy(), g[f"{name}_grad"], rtol=1e-5, atol=1e-9)


def test_positional_encoding():
    g = golden("nerf.npz")
    pts, dirs = torch.from_numpy(g["pe_pts"]), torch.from_numpy(g["pe_dirs"])
    assert torch.equal(ref_path.positional_encoding(pts, [14, 14, 10]), torch.from_numpy(g["pe_list"]))
    assert torch.equal(ref_path.positional_encoding(dirs, 4), torch.from_numpy(g["pe_int"]))
