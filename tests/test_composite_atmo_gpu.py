"""K8 (csrc/composite.hip) in the atmospheric regime, against the REFERENCE's own output.

tests/golden/render_atmo.npz: the reference's render_with_surface (graphics_utils.py:
6-77) run by oracle/gen_golden.py on f64 tensors (its formula evaluated exactly) and on
f32 tensors, at BASELINE configs[2]'s 1,024 samples per ray over 22.7 km with
sigma in [1e-5, 2e-4] km^-1 -- the synthetic atmosphere at initialisation, where
1 - exp(-sigma * delta) cancels in f32. K8 (f32, alpha = -expm1(-x), d alpha/dx = exp(-x))
must hold alpha, weights, the three colour maps and dL/d{color, sigma, color_surf, z} for
a loss on color_map within 1e-4 of the reference-f64 values (relative to each quantity's
largest magnitude). The reference's own f32 evaluation is measured against the same f64
values and recorded beside it (ANR_COMPOSITE_ATMO_OUT).
"""

import json
import os

import numpy as np
import pytest
import torch

from tests.conftest import golden

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def test_composite_matches_reference_f64_in_atmosphere(dev):
    from atmonr_amd import _lib

    d = golden("render_atmo.npz")
    B, N, C = d["color"].shape
    t = lambda k: torch.from_numpy(d[k]).float().to(dev).contiguous()  # noqa: E731
    z, color, sigma, cs, gcm = t("z"), t("color"), t("sigma"), t("cs"), t("gcm")
    cm = torch.empty(B, C, device=dev)
    atmo, surf = torch.empty_like(cm), torch.empty_like(cm)
    w = torch.empty(B, N, 1, device=dev)
    alpha = torch.empty_like(w)
    s = _lib.stream(dev)
    ptr = _lib.ptr
    _lib.call("anr_composite_fwd", ptr(z), 1.0, ptr(color), ptr(sigma), ptr(cs), _lib.F32, B, N,
              C, 1, ptr(cm), ptr(atmo), ptr(surf), ptr(w), ptr(alpha), s)
    dcol, dsig, dcs = torch.empty_like(color), torch.empty_like(sigma), torch.empty_like(cs)
    dz = torch.empty(B, N, device=dev)
    _lib.call("anr_composite_bwd", ptr(z), 1.0, ptr(color), ptr(sigma), ptr(cs), _lib.F32, B, N,
              C, 1, ptr(gcm), None, None, None, None, ptr(dcol), ptr(dsig), ptr(dcs), ptr(dz), s)
    got = {"cm": cm, "alpha": alpha, "w": w, "atmo": atmo, "surf": surf, "dcolor": dcol,
           "dsigma": dsig, "dcs": dcs, "dz": dz}
    rec = {}
    for k, v in got.items():
        ref64 = d["f64_" + k].reshape(tuple(v.shape))
        rec[k] = {"k8_vs_f64": _rel(v.double().cpu().numpy(), ref64),
                  "reference_f32_vs_f64": _rel(d["f32_" + k].reshape(ref64.shape), ref64)}
    out = os.environ.get("ANR_COMPOSITE_ATMO_OUT")
    if out:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as f:
            json.dump(rec, f, indent=1)
    for k, r in rec.items():
        assert r["k8_vs_f64"] <= 1e-4, (k, rec)
