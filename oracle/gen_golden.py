"""Generate golden vectors by RUNNING THE REFERENCE (build container only).

    PYTHONPATH=/root/reference/src python oracle/gen_golden.py   # writes tests/golden/*.npz

The reference package ``atmonr`` is imported from /root/reference/src (read-only). Its
dataset module imports netCDF4 / h5py / earthaccess / torchmetrics at module level; those
are I/O / metrics libraries absent here and are stubbed in sys.modules (only the pure
functions below are called). Each fixture stores inputs and the reference's outputs;
nothing from the reference's source travels with the repo.
"""

from __future__ import annotations

import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = os.environ.get("ATMONR_REF", "/root/reference/src")
OUT = Path(__file__).resolve().parent.parent / "tests" / "golden"


def _stub_modules():
    for name in ["netCDF4", "h5py", "earthaccess", "torchmetrics", "torchmetrics.functional",
                 "torchmetrics.functional.image"]:
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
    img = sys.modules["torchmetrics.functional.image"]
    img.peak_signal_noise_ratio = None
    img.structural_similarity_index_measure = None
    sys.modules["netCDF4"].Dataset = object
    sys.modules["netCDF4"].Variable = object


def main():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    _stub_modules()
    from atmonr import encoders, graphics_utils, losses, samplers  # noqa: E402
    from atmonr.datasets.harp2 import HARP2Dataset  # noqa: E402
    from atmonr.geospatial import wgs_84  # noqa: E402
    from atmonr.models.nerf import AtmoNeRF  # noqa: E402

    OUT.mkdir(parents=True, exist_ok=True)
    g = torch.Generator().manual_seed(1234)

    # --- sample_uniform_bins (samplers.py:8-47) --------------------------------------
    fx = {}
    for tag, B, N in [("a", 97, 64), ("b", 8, 1024), ("c", 5, 7)]:
        origin = torch.rand(B, 3, generator=g) * 2 - 1
        direction = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=1)
        length = torch.rand(B, generator=g) * 1.5 + 0.1
        batch = {"origin": origin, "dir": direction, "len": length}
        torch.manual_seed(100 + B)
        pts, z = samplers.sample_uniform_bins(batch, N)
        torch.manual_seed(100 + B)
        u = torch.rand((B, N))
        pts_mid, z_mid = samplers.sample_uniform_bins(batch, N, random=False)
        fx.update({f"{tag}_origin": origin, f"{tag}_dir": direction, f"{tag}_len": length,
                   f"{tag}_u": u, f"{tag}_pts": pts, f"{tag}_z": z, f"{tag}_pts_mid": pts_mid,
                   f"{tag}_z_mid": z_mid})
    np.savez_compressed(OUT / "sampler.npz", **{k: v.numpy() for k, v in fx.items()})

    # --- horizontal point preprocessor (harp2.py:357-388) -----------------------------
    fx = {}
    for tag, (lat0, lon0) in [("std", (30.0, -60.0)), ("dateline", (-10.0, 179.9))]:
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
        fake = types.SimpleNamespace(lat=lat, lon=lon, scale=scale, offset=offset,
                                     config={"ray_origin_height": 20000})
        prep = HARP2Dataset.get_point_preprocessor(fake, "horizontal")
        batch = {"origin": o_n, "dir": d, "len": ln / scale}
        torch.manual_seed(7)
        pts, z = samplers.sample_uniform_bins(batch, 32)
        coords = prep(pts)
        la, lo = lat[~lat.isnan()], lon[~lon.isnan()]
        lat_min, lat_max, lon_min, lon_max = la.min(), la.max(), lo.min(), lo.max()
        shift = bool(lon_max > 179 and lon_min < -179)
        if shift:
            lo2 = lo % 360 - 180
            lon_min, lon_max = lo2.min(), lo2.max()
        fx.update({
            f"{tag}_pts": pts, f"{tag}_coords": coords,
            f"{tag}_meta": torch.tensor([scale, float(lat_min), float(lat_max - lat_min),
                                         float(lon_min), float(lon_max - lon_min), 20000.0,
                                         float(shift)], dtype=torch.float64),
            f"{tag}_offset": offset.double(),
            f"{tag}_ray_origin": o_n, f"{tag}_ray_dir": d, f"{tag}_ray_len": ln / scale,
        })
        # cartesian_to_horizontal itself (wgs_84.py:56-97)
        xyz = pts.reshape(-1, 3).double() * scale + offset
        la2, lo2_, al2 = wgs_84.cartesian_to_horizontal(xyz[:, 0], xyz[:, 1], xyz[:, 2])
        fx[f"{tag}_c2h"] = torch.stack([la2, lo2_, al2], dim=1)
    np.savez_compressed(OUT / "preprocess.npz", **{k: v.numpy() for k, v in fx.items()})

    # --- render / render_with_surface + autograd (graphics_utils.py:6-77) ------------
    fx = {}
    for tag, B, N, C, S, dt in [("f32", 16, 64, 4, 1, torch.float32),
                                ("f32long", 4, 1024, 4, 1, torch.float32),
                                ("f32multi", 8, 48, 4, 4, torch.float32),
                                ("f16", 16, 64, 4, 1, torch.float16)]:
        z = (torch.sort(torch.rand(B, N, generator=g), dim=1)[0] * 22.0).float()
        color = (torch.rand(B, N, C, generator=g) * 2).to(dt)
        sigma = (torch.rand(B, N, S, generator=g) * 0.8).to(dt)
        sigma[:, : N // 8] = 0  # clear air
        sigma[0, N // 2] = 40.0  # an almost opaque sample
        cs = (torch.rand(B, C, generator=g)).to(dt)
        gcm = torch.randn(B, C, generator=g).to(dt)
        gatmo = torch.randn(B, C, generator=g).to(dt)
        gsurf = torch.randn(B, C, generator=g).to(dt)
        gw = (torch.randn(B, N, S, generator=g) * 0.1).to(dt)
        zz = z.clone().requires_grad_(True)
        cc = color.clone().requires_grad_(True)
        ss = sigma.clone().requires_grad_(True)
        css = cs.clone().requires_grad_(True)
        cm, alpha, w, atmo, surf = graphics_utils.render_with_surface(zz, cc, ss, css)
        loss = (cm * gcm).sum() + (atmo * gatmo).sum() + (surf * gsurf).sum() + (w * gw).sum()
        loss.backward()
        fx.update({f"{tag}_z": z, f"{tag}_color": color, f"{tag}_sigma": sigma,
                   f"{tag}_cs": cs, f"{tag}_gcm": gcm, f"{tag}_gatmo": gatmo,
                   f"{tag}_gsurf": gsurf, f"{tag}_gw": gw, f"{tag}_cm": cm.detach(),
                   f"{tag}_alpha": alpha.detach(), f"{tag}_w": w.detach(),
                   f"{tag}_atmo": atmo.detach(), f"{tag}_surf": surf.detach(),
                   f"{tag}_dz": zz.grad, f"{tag}_dcolor": cc.grad, f"{tag}_dsigma": ss.grad,
                   f"{tag}_dcs": css.grad})
        cm2, a2, w2 = graphics_utils.render(z, color, sigma)
        fx.update({f"{tag}_plain_cm": cm2, f"{tag}_plain_w": w2})
    np.savez_compressed(OUT / "render.npz",
                        **{k: v.float().numpy() if v.dtype == torch.float16 else v.numpy()
                           for k, v in fx.items()})

    # --- losses (losses.py:5-33) -------------------------------------------------------
    fx = {}
    B = 257
    pred = torch.rand(B, generator=g) * 50 + 1e-3
    gt = torch.rand(B, generator=g) * 50
    max_i = 61.5
    fx["pred"], fx["gt"], fx["max_i"] = pred, gt, torch.tensor(max_i)
    for name in ["dark", "hdr", "l1", "l1_plus_hdr", "mse", "mse_plus_hdr"]:
        p = pred.clone().requires_grad_(True)
        val = getattr(losses, f"{name}_loss")(p, gt, max_i)
        val.backward()
        fx[f"{name}_val"], fx[f"{name}_grad"] = val.detach(), p.grad
    np.savez_compressed(OUT / "losses.npz", **{k: v.numpy() for k, v in fx.items()})

    # --- positional encoding + a small AtmoNeRF (encoders.py, models/nerf.py) ---------
    fx = {}
    pts = torch.rand(3, 11, 3, generator=g) * 2 - 1
    dirs = torch.nn.functional.normalize(torch.randn(3, 11, 3, generator=g), dim=-1)
    fx["pe_pts"], fx["pe_dirs"] = pts, dirs
    fx["pe_list"] = encoders.positional_encoding(pts, [14, 14, 10])
    fx["pe_int"] = encoders.positional_encoding(dirs, 4)
    torch.manual_seed(3)
    net = AtmoNeRF(pos_channels=76, dir_channels=24, out_channels=4, volume_channels=1,
                   hidden_dim=32).eval()
    x = torch.randn(40, 100, generator=g)
    color, sigma = net(x)
    fx["nerf_x"], fx["nerf_color"], fx["nerf_sigma"] = x, color.detach(), sigma.detach()
    for k, v in net.state_dict().items():
        fx[f"nerf_w_{k}"] = v
    np.savez_compressed(OUT / "nerf.npz", **{k: v.numpy() for k, v in fx.items()})

    # --- sample_pdf (samplers.py:50-103) ------------------------------------------------
    fx = {}
    B, Nc = 6, 64
    origin = torch.rand(B, 3, generator=g) * 2 - 1
    direction = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=1)
    zc = torch.sort(torch.rand(B, Nc, generator=g), dim=1)[0] * 1.3
    wts = torch.rand(B, Nc, 1, generator=g)
    wts[0, 5:20] = 0
    batch = {"origin": origin, "dir": direction}
    torch.manual_seed(11)
    pts, z = samplers.sample_pdf(batch, wts, zc, n_samples=128)
    torch.manual_seed(11)
    u = torch.rand(B, 128)
    fx.update(dict(origin=origin, dir=direction, zc=zc, w=wts, u=u, pts=pts, z=z))
    np.savez_compressed(OUT / "sample_pdf.npz", **{k: v.numpy() for k, v in fx.items()})

    # --- render_with_surface in the atmospheric regime (r03) ---------------------------
    # sigma in [1e-5, 2e-4] km^-1, 1,024 samples up to 22.7 km (BASELINE configs[2]'s
    # rays at initialisation): the reference's own function on f64, f32 and f16 tensors,
    # with dL/d{color, sigma, color_surf} for a loss on color_map alone (the training
    # loss's path). graphics_utils.py:28 casts z to color.dtype, so the f64 run is the
    # reference's formula evaluated exactly.
    g3 = torch.Generator().manual_seed(2026)
    fx = {}
    B, N, C = 6, 1024, 4
    z = (torch.sort(torch.rand(B, N, generator=g3, dtype=torch.float64), dim=1)[0] * 22.7)
    color = torch.rand(B, N, C, generator=g3, dtype=torch.float64)
    sigma = torch.exp(torch.empty(B, N, 1, dtype=torch.float64).uniform_(
        np.log(1e-5), np.log(2e-4), generator=g3))
    cs = torch.rand(B, C, generator=g3, dtype=torch.float64)
    gcm = torch.randn(B, C, generator=g3, dtype=torch.float64) * 1e-3
    fx.update(z=z, color=color, sigma=sigma, cs=cs, gcm=gcm)
    for tag, dt in [("f64", torch.float64), ("f32", torch.float32), ("f16", torch.float16)]:
        cc = color.detach().clone().to(dt).requires_grad_(True)
        ss = sigma.detach().clone().to(dt).requires_grad_(True)
        css = cs.detach().clone().to(dt).requires_grad_(True)
        zz = z.float() if dt == torch.float16 else z.to(dt)  # the f16 path gets f32 z
        zz = zz.detach().clone().requires_grad_(dt != torch.float16)
        cm, alpha, w, atmo, surf = graphics_utils.render_with_surface(zz, cc, ss, css)
        cm.backward(gcm.to(dt))
        fx.update({f"{tag}_cm": cm.detach(), f"{tag}_alpha": alpha.detach(),
                   f"{tag}_w": w.detach(), f"{tag}_atmo": atmo.detach(),
                   f"{tag}_surf": surf.detach(), f"{tag}_dcolor": cc.grad,
                   f"{tag}_dsigma": ss.grad, f"{tag}_dcs": css.grad})
        if dt != torch.float16:
            fx[f"{tag}_dz"] = zz.grad
        if dt == torch.float16:  # the surface product (graphics_utils.py:75) on its own
            fx["f16_pr"] = (1 - alpha.detach()).prod(dim=1)
    np.savez_compressed(OUT / "render_atmo.npz",
                        **{k: v.double().numpy() for k, v in fx.items()})

    # --- the f16 composite and loss the reference's Instant-NGP step runs (r03) ---------
    # f16 tensors into render_with_surface and mse_plus_hdr etc., gradients through
    # color_map / the prediction only: the reference's f16 autograd on CPU torch
    fx = {}
    for tag, B, N, smax in [("a", 12, 64, 1.0), ("b", 4, 1024, 2e-3)]:
        z = torch.sort(torch.rand(B, N, generator=g3), dim=1)[0] * 22.7
        color = torch.rand(B, N, 4, generator=g3).half().requires_grad_(True)
        sigma = (torch.rand(B, N, 1, generator=g3) * smax).half().requires_grad_(True)
        cs = torch.rand(B, 4, generator=g3).half().requires_grad_(True)
        gcm = (torch.randn(B, 4, generator=g3) * 1e-3).half()
        cm, alpha, w, atmo, surf = graphics_utils.render_with_surface(z, color, sigma, cs)
        cm.backward(gcm)
        fx.update({f"{tag}_z": z, f"{tag}_color": color.detach(), f"{tag}_sigma": sigma.detach(),
                   f"{tag}_cs": cs.detach(), f"{tag}_gcm": gcm, f"{tag}_cm": cm.detach(),
                   f"{tag}_alpha": alpha.detach(), f"{tag}_w": w.detach(),
                   f"{tag}_atmo": atmo.detach(), f"{tag}_surf": surf.detach(),
                   f"{tag}_pr": (1 - alpha.detach()).prod(dim=1),
                   f"{tag}_dcolor": color.grad, f"{tag}_dsigma": sigma.grad,
                   f"{tag}_dcs": cs.grad})
    B = 256
    pred = (torch.rand(B, generator=g3) * 0.3).half()
    gt = (torch.rand(B, generator=g3) * 0.3)
    for mi in (0.37, 61.5):
        for name in ["dark", "hdr", "l1", "l1_plus_hdr", "mse", "mse_plus_hdr"]:
            p = pred.clone().requires_grad_(True)
            val = getattr(losses, f"{name}_loss")(p, gt.half(), mi)
            val.backward()
            fx[f"loss_{mi}_{name}_val"], fx[f"loss_{mi}_{name}_grad"] = val.detach(), p.grad
    fx["loss_pred"], fx["loss_gt"] = pred, gt
    np.savez_compressed(OUT / "f16_step.npz",
                        **{k: v.float().numpy() if v.dtype == torch.float16 else v.numpy()
                           for k, v in fx.items()})
    print("golden vectors written to", OUT)
    for f in sorted(OUT.glob("*.npz")):
        print(f"  {f.name}: {f.stat().st_size / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
