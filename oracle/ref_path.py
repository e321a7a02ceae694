"""ORACLE (test infrastructure only): CPU restatement of the AtmoNR hot path pieces that
live in the reference itself. Each function cites the reference lines it follows and is
pinned against golden vectors produced by the reference (tests/golden/*.npz).
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

WGS_A = 6378137.0
WGS_B = 6356752.314245
WGS_E = (WGS_A**2 - WGS_B**2) / (WGS_A**2)
WGS_E2 = (WGS_A**2 - WGS_B**2) / (WGS_B**2)


# ---------------------------------------------------------------- samplers.py:8-47
def sample_uniform_bins(origin, direction, length, u=None, n_bins=64):
    """Stratified samples; u (B, n_bins) f32 or None for bin midpoints."""
    bins = torch.linspace(0, 1, n_bins + 1)[None]
    t = u if u is not None else 0.5
    z = (bins[:, :-1] + t / n_bins) * length[:, None]
    pts = origin[:, None] + direction[:, None] * z[..., None]
    return pts, z


# ---------------------------------------------------------------- harp2.py:357-388
def preprocess_horizontal(pts: np.ndarray, scale, offset, lat_min, lat_range, lon_min,
                          lon_range, h0, shift_lon=False) -> np.ndarray:
    """pts (..., 3) f32 -> (..., 3) f32 via Bowring (wgs_84.py:56-97) in float64."""
    p = pts.astype(np.float32) * np.float32(scale)  # f32 tensor * Python float
    xyz = p.astype(np.float64) + np.asarray(offset, dtype=np.float64)
    x, y, z = xyz[..., 0], xyz[..., 1], xyz[..., 2]
    lon = np.arctan2(y, x)
    D = np.sqrt(x * x + y * y)
    u = np.arctan2(z / D, np.zeros_like(x) + WGS_A / WGS_B)
    su, cu = np.sin(u), np.cos(u)
    lat = np.arctan2(z + (WGS_E2 * WGS_B) * (su * su * su), D - (WGS_E * WGS_A) * (cu * cu * cu))
    sl = np.sin(lat)
    Nr = WGS_A / np.sqrt(1 - WGS_E * (sl * sl))
    alt = x / (np.cos(lat) * np.cos(lon)) - Nr
    lat = lat * 180 / math.pi
    lon = lon * 180 / math.pi
    if shift_lon:
        lon = np.mod(lon, 360) - 180
    a = 2 * (lat - lat_min) / lat_range - 1
    b = 2 * (lon - lon_min) / lon_range - 1
    c = 2 * alt / h0 - 1
    out = np.stack([a, b, c], axis=-1).astype(np.float32)
    return np.clip(out, -1, 1)


# ---------------------------------------------------------------- graphics_utils.py:6-77
def render(z, color, sigma):
    z = z.to(dtype=color.dtype)
    mid = (z[..., :-1] + z[..., 1:]) / 2
    mid = torch.cat([z[..., :1] * 0, mid, z[..., -1:]], dim=-1)
    delta = torch.diff(mid, dim=-1)[..., None]
    alpha = 1 - torch.exp(-sigma * delta)
    ones = torch.ones((alpha.shape[0], 1, alpha.shape[2]), dtype=alpha.dtype)
    weights = alpha * torch.cumprod(torch.cat([ones, 1 - alpha + 1e-10], dim=1), dim=1)[:, :-1]
    return torch.sum(color * weights, dim=1), alpha, weights


def render_with_surface(z, color, sigma, color_surf):
    atmo, alpha, weights = render(z, color, sigma)
    surf = (1 - alpha).prod(dim=1) * color_surf
    return atmo + surf, alpha, weights, atmo, surf


# ---------------------------------------------------------------- losses.py:5-33
def _hdr(p, g, m):
    return F.mse_loss(torch.log(g + 1e-3 * m), torch.log(p + 1e-3 * m))


LOSSES = {
    "dark": lambda p, g, m: (((p - g) / (p.detach() + 1e-3 * m)) ** 2).mean(),
    "hdr": _hdr,
    "l1": lambda p, g, m: F.l1_loss(p / m, g / m),
    "l1_plus_hdr": lambda p, g, m: F.l1_loss(p / m, g / m) + 0.2 * _hdr(p, g, m),
    "mse": lambda p, g, m: F.mse_loss(p / m, g / m),
    "mse_plus_hdr": lambda p, g, m: F.mse_loss(p / m, g / m) + 0.2 * _hdr(p, g, m),
}


# ---------------------------------------------------------------- encoders.py:4-28
def positional_encoding(pts, L):
    if isinstance(L, int):
        p = pts.reshape(-1, pts.shape[-1])[..., None, None]
        ls = torch.linspace(0, L - 1, steps=L)
        ls = torch.stack([ls, ls], dim=1)
        p = (2**ls * torch.pi)[None, None] * p
        p = torch.stack([torch.sin(p[..., 0]), torch.cos(p[..., 1])], dim=-1)
        return p.reshape(p.shape[0], p.shape[1], -1)
    outs = []
    for i, n in enumerate(L):
        ls = torch.linspace(0, n - 1, steps=n)
        x = (2**ls * torch.pi)[..., None, :] * pts[..., i, None]
        outs.append(torch.cat([torch.sin(x), torch.cos(x)], dim=-1))
    return torch.cat(outs, dim=-1)
