"""The f16 restatement (oracle/ref_f16.py) pinned to the reference's own f16 outputs.

tests/golden/f16_step.npz holds what the REFERENCE computes (oracle/gen_golden.py runs
src/atmonr/graphics_utils.py and losses.py on f16 tensors, torch on the CPU): the
composite's outputs and its f16 autograd for a loss on color_map, and the six losses with
their gradients. ref_f16 in its CPU form (acc="cpu") must reproduce every value BIT FOR
BIT -- that pins each rounding point and autograd's accumulation order. torch's CPU prod
over f16 is not restated (it accumulates in f16 lanes); those tests take the reference's
own product (``*_pr``) as input. tests/golden/render_atmo.npz (the reference on f64 / f32
/ f16 tensors in the atmospheric regime) pins ref_path's f64 composite.
"""

import numpy as np
import pytest
import torch

from oracle import ref_f16, ref_path
from tests.conftest import golden


@pytest.mark.parametrize("tag", ["a", "b"])
def test_composite_cpu_form_matches_reference_bitwise(tag):
    d = golden("f16_step.npz")
    r = ref_f16.render_fwd(d[f"{tag}_z"].astype(np.float32), d[f"{tag}_color"],
                           d[f"{tag}_sigma"], d[f"{tag}_cs"], acc="cpu",
                           prod_override=d[f"{tag}_pr"])
    for k, ref in [("color_map", "cm"), ("alpha", "alpha"), ("w", "w"), ("atmo", "atmo"),
                   ("surf", "surf")]:
        assert np.array_equal(r[k], d[f"{tag}_{ref}"].reshape(r[k].shape)), k
    gb = ref_f16.render_bwd(r, d[f"{tag}_gcm"], acc="cpu")
    for k, ref in [("color", "dcolor"), ("sigma", "dsigma"), ("cs", "dcs")]:
        want = d[f"{tag}_{ref}"].reshape(gb[k].shape)
        assert np.array_equal(gb[k], want), (k, int((gb[k] != want).sum()))


@pytest.mark.parametrize("mi", [0.37, 61.5])
@pytest.mark.parametrize("name", ["dark", "hdr", "l1", "l1_plus_hdr", "mse", "mse_plus_hdr"])
def test_loss_cpu_form_matches_reference_bitwise(mi, name):
    d = golden("f16_step.npz")
    gt16 = d["loss_gt"].astype(np.float16).astype(np.float32)
    v, g = ref_f16.loss_f16(name, d["loss_pred"], gt16, mi, acc="cpu")
    assert np.array_equal(g, d[f"loss_{mi}_{name}_grad"])
    assert float(v) == float(d[f"loss_{mi}_{name}_val"])


def test_cuda_form_differs_only_by_accumulation():
    # the same inputs through the CUDA form: the elementwise path is identical, the f16
    # accumulator of cumprod moves the transmittance
    d = golden("f16_step.npz")
    args = (d["a_z"].astype(np.float32), d["a_color"], d["a_sigma"], d["a_cs"])
    cpu = ref_f16.render_fwd(*args, acc="cpu", prod_override=d["a_pr"])
    cuda = ref_f16.render_fwd(*args, acc="cuda")
    assert np.array_equal(cpu["alpha"], cuda["alpha"])
    assert not np.array_equal(cpu["T"], cuda["T"])


def test_oracle_composite_f64_matches_reference_atmospheric_regime():
    d = golden("render_atmo.npz")
    t = {k: torch.from_numpy(d[k]) for k in ("z", "color", "sigma", "cs", "gcm")}
    z = t["z"].clone().requires_grad_(True)
    c = t["color"].clone().requires_grad_(True)
    s = t["sigma"].clone().requires_grad_(True)
    cs = t["cs"].clone().requires_grad_(True)
    cm, alpha, w, atmo, surf = ref_path.render_with_surface(z, c, s, cs)
    cm.backward(t["gcm"])
    for got, key in [(cm, "f64_cm"), (alpha, "f64_alpha"), (w, "f64_w"), (atmo, "f64_atmo"),
                     (surf, "f64_surf"), (c.grad, "f64_dcolor"), (s.grad, "f64_dsigma"),
                     (cs.grad, "f64_dcs"), (z.grad, "f64_dz")]:
        assert np.array_equal(got.detach().numpy(), d[key]), key


def test_cuda_loss_adds_scalar_in_f32():
    # x + 1e-3 * max_i: torch on CUDA adds the Python scalar in f32, on the CPU rounded to
    # f16 first -- the two forms differ exactly there
    p = ref_f16.h(np.linspace(0.01, 0.3, 64))
    g = ref_f16.h(np.linspace(0.3, 0.01, 64))
    _, g_cpu = ref_f16.loss_f16("hdr", p, g, 0.37, acc="cpu")
    _, g_cuda = ref_f16.loss_f16("hdr", p, g, 0.37, acc="cuda")
    assert not np.array_equal(g_cpu, g_cuda)
    _, m_cpu = ref_f16.loss_f16("mse", p, g, 0.37, acc="cpu")
    _, m_cuda = ref_f16.loss_f16("mse", p, g, 0.37, acc="cuda")
    assert np.array_equal(m_cpu, m_cuda)
