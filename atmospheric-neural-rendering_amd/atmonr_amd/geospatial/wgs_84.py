"""WGS-84 geometry used to build HARP2-shaped ray sets (scene setup, not the hot loop).

Same conventions as src/atmonr/geospatial/wgs_84.py: EPSG:4326 <-> EPSG:4978 and the
normalized scene frame. The per-sample hot-path conversion (Bowring's
cartesian_to_horizontal inside the point preprocessor, wgs_84.py:56-97) runs in the K2
HIP kernel (csrc/sampler.hip); the torch versions here serve ray construction
(get_rays, wgs_84.py:223-290), filtering (:293-313) and normalization (:316-339), which
run once per scene.
"""

from __future__ import annotations

import math

import torch

A = 6378137.0
B = 6356752.314245
E = (A * A - B * B) / (A * A)     # first eccentricity squared
E2 = (A * A - B * B) / (B * B)    # second eccentricity squared


def horizontal_to_cartesian(lat, lon, alt):
    """(lat, lon in degrees, ellipsoidal height m) -> WGS-84 Cartesian (x, y, z), with
    the reference's operation order (wgs_84.py:24-53), so f64 results match bit for bit."""
    phi, lam = lat * math.pi / 180, lon * math.pi / 180
    sphi = torch.sin(phi)
    n = A / torch.sqrt(1 - (E * sphi ** 2))
    r = (n + alt) * torch.cos(phi)
    return r * torch.cos(lam), r * torch.sin(lam), (n * (1 - E) + alt) * sphi


def cartesian_to_horizontal(x, y, z):
    """Bowring's one-step inverse; returns (lat deg, lon deg, height m)."""
    lon = torch.atan2(y, x)
    p = torch.sqrt(x * x + y * y)
    beta = torch.atan2(z / p, torch.full_like(x, A / B))
    sb, cb = torch.sin(beta), torch.cos(beta)
    lat = torch.atan2(z + E2 * B * sb ** 3, p - E * A * cb ** 3)
    sl = torch.sin(lat)
    n = A / torch.sqrt(1 - (E * sl ** 2))
    alt = x / (torch.cos(lat) * torch.cos(lon)) - n
    return lat * 180 / math.pi, lon * 180 / math.pi, alt


def _rotation(theta_deg, phi_deg):
    """Rotation built from (zenith, azimuth) in degrees; same sense as the reference."""
    t, p = -theta_deg * math.pi / 180, -phi_deg * math.pi / 180
    st, ct, sp, cp = torch.sin(t), torch.cos(t), torch.sin(p), torch.cos(p)
    zero = torch.zeros_like(t)
    row0 = torch.stack([cp, -sp * ct, sp * st], dim=-1)
    row1 = torch.stack([sp, cp * ct, -cp * st], dim=-1)
    row2 = torch.stack([zero, st, ct], dim=-1)
    return torch.stack([row0, row1, row2], dim=-2)


def view_directions(thetav, phiv):
    """Unit view vectors in the local (+x east, +y north, +z up) frame."""
    up = torch.zeros(thetav.shape + (3,), dtype=thetav.dtype, device=thetav.device)
    up[..., 2] = 1.0
    return (_rotation(thetav, phiv) @ up[..., None])[..., 0]


def local_to_ecef(dirs, lat, lon):
    """Rotate local-frame vectors at (lat, lon) into the WGS-84 Cartesian frame."""
    rot = _rotation(90.0 - lat, 90.0 - lon).to(dirs.dtype)
    flip = torch.tensor([[-1.0, 0, 0], [0, -1.0, 0], [0, 0, 1.0]], dtype=dirs.dtype,
                        device=dirs.device)
    return (rot @ (flip @ dirs[..., None]))[..., 0]


def get_rays(lat, lon, alt, thetav, phiv, ray_origin_height, tol=10.0, max_iters=20):
    """Ray origins at `ray_origin_height`, directions toward the surface and lengths.

    Follows the reference formulation (wgs_84.py:223-290): the surface point in fp64,
    the view vector rotated into ECEF and flipped, then an iterative rescale of the
    length until the origin's ellipsoidal height is within `tol` metres.
    """
    x, y, z = horizontal_to_cartesian(lat.double(), lon.double(), alt.double())
    surf = torch.stack([x, y, z], dim=-1).float()
    d = local_to_ecef(view_directions(thetav.double(), phiv.double()).reshape(-1, 3),
                      lat.reshape(-1), lon.reshape(-1))
    d = -d.view(surf.shape)
    lens = (ray_origin_height - alt) / torch.cos(thetav * math.pi / 180).double()

    def height(lens):
        o = surf - lens[..., None] * d
        return cartesian_to_horizontal(o[..., 0], o[..., 1], o[..., 2])[2]

    h = height(lens)
    it = 0
    while it < max_iters and (torch.abs(ray_origin_height - h) > tol).any():
        lens = lens * ray_origin_height / h
        h = height(lens)
        it += 1
    lens = lens.float()
    origins = (surf - d * lens[..., None]).reshape(-1, 3)
    return origins.float(), d.reshape(-1, 3).float(), lens.reshape(-1).float()


def filter_rays(origin, direction, rad):
    """Valid-ray mask: finite origin, direction and radiance (wgs_84.py:293-313)."""
    return ~(origin.isnan().any(1) | direction.isnan().any(1) | rad.isnan())


def normalize_rays(origin, direction, length):
    """Map the scene into [-1, 1]^3; returns (origin_norm, scale, offset) (wgs_84.py:316)."""
    ends = origin + direction * length[:, None]
    pts = torch.cat([origin, ends], dim=0)
    hi = pts.max(dim=0)[0].double()
    lo = pts.min(dim=0)[0].double()
    scale = ((hi - lo).max() / 2).item()
    offset = (hi + lo) / 2
    return torch.clamp((origin - offset) / scale, -1, 1).float(), scale, offset
