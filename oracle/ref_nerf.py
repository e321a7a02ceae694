"""ORACLE (test infrastructure only): the configs/nerf.json train step restated on CPU.

Used as bench.py's ``cpu_baseline`` ("port") and pinned by tests/test_oracle_nerf.py
against golden vectors from the reference (AtmoNeRF forward, sample_pdf, positional
encoding). Follows:
  NeRFPipeline._forward / forward / compute_loss   src/atmonr/pipelines/nerf.py:73-240
  AtmoNeRF / get_model                             src/atmonr/models/nerf.py:6-144
  sample_uniform_bins / sample_pdf                 src/atmonr/samplers.py:8-103
  preprocess_coords (torch, differentiable)        src/atmonr/datasets/harp2.py:372-386
  render                                           src/atmonr/graphics_utils.py:6-49
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from oracle.ref_path import WGS_A, WGS_B, WGS_E, WGS_E2, positional_encoding, render


class RefAtmoNeRF(nn.Module):
    """models/nerf.py:6-93: 11 Linear layers, skip at fc6, density head at fc9."""

    def __init__(self, pos_channels, dir_channels, out_channels, volume_channels, hidden=256):
        super().__init__()
        h = hidden
        self.pos_channels, self.hidden_dim = pos_channels, h
        dims = [(pos_channels, h), (h, h), (h, h), (h, h), (h, h), (h + pos_channels, h),
                (h, h), (h, h), (h, h + volume_channels), (h + dir_channels, h // 2),
                (h // 2, out_channels)]
        for i, (a, b) in enumerate(dims, start=1):
            setattr(self, f"fc{i}", nn.Linear(a, b))
            nn.init.kaiming_normal_(getattr(self, f"fc{i}").weight, mode="fan_out")

    def forward_pos_only(self, x_pos):
        x = x_pos
        for i in range(1, 6):
            x = F.relu(getattr(self, f"fc{i}")(x))
        x = torch.cat([x, x_pos], dim=1)
        for i in range(6, 9):
            x = F.relu(getattr(self, f"fc{i}")(x))
        x = self.fc9(x)
        sigma = x[:, self.hidden_dim:]
        if self.training:
            sigma = sigma + torch.randn(sigma.shape)
        return x, F.relu(sigma)

    def forward(self, x):
        x_pos, d = x[:, : self.pos_channels], x[:, self.pos_channels:]
        x, sigma = self.forward_pos_only(x_pos)
        x = F.relu(self.fc10(torch.cat([x[:, : self.hidden_dim], d], dim=1)))
        return torch.sigmoid(self.fc11(x)), sigma


def sample_uniform(origin, direction, length, n_bins):
    bins = torch.linspace(0, 1, n_bins + 1)[None]
    z = (bins[:, :-1] + torch.rand(origin.shape[0], n_bins) / n_bins) * length[:, None]
    return origin[:, None] + direction[:, None] * z[..., None], z


def sample_pdf(origin, direction, weights, z_c, n_samples, u=None):
    """samplers.py:50-103 (gradients reach `weights` through t_in_bin)."""
    pdf = weights[:, 1:-1, 0] + 1e-8
    pdf = pdf / torch.sum(pdf, dim=1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, dim=1)], dim=1)
    if u is None:
        u = torch.rand(list(cdf.shape[:-1]) + [n_samples])
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.clamp(inds - 1, min=0)
    above = torch.clamp(inds, max=cdf.shape[-1] - 1)
    ig = torch.stack([below, above], -1)
    mid = 0.5 * (z_c[..., 1:] + z_c[..., :-1])
    shp = [ig.shape[0], ig.shape[1], cdf.shape[-1]]
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(shp), 2, ig)
    bins_g = torch.gather(mid.unsqueeze(1).expand(shp), 2, ig)
    denom = cdf_g[..., 1] - cdf_g[..., 0]
    denom = torch.where(denom < 1e-8, torch.ones_like(denom), denom)
    t = (u - cdf_g[..., 0]) / denom
    samples = bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0]).detach()
    z, _ = torch.sort(torch.cat([z_c, samples], -1), -1)
    return origin[:, None] + direction[:, None] * z[..., None], z


def preprocess_torch(pts, scale, offset, lat_min, lat_range, lon_min, lon_range, h0,
                     shift_lon=False):
    """Differentiable harp2.py:372-386 in float64 torch (NeRF back-propagates through it)."""
    dtype = pts.dtype
    xyz = pts * scale + offset
    x, y, z = xyz[..., 0], xyz[..., 1], xyz[..., 2]
    lon = torch.atan2(y, x)
    D = torch.sqrt(x**2 + y**2)
    u = torch.atan2(z / D, torch.zeros_like(x) + WGS_A / WGS_B)
    lat = torch.atan2(z + (WGS_E2 * WGS_B) * torch.sin(u) ** 3,
                      D - (WGS_E * WGS_A) * torch.cos(u) ** 3)
    Nr = WGS_A / torch.sqrt(1 - WGS_E * torch.sin(lat) ** 2)
    alt = x / (torch.cos(lat) * torch.cos(lon)) - Nr
    lat = lat * 180 / math.pi
    lon = lon * 180 / math.pi
    if shift_lon:
        lon = lon % 360 - 180
    lat = 2 * (lat - lat_min) / lat_range - 1
    lon = 2 * (lon - lon_min) / lon_range - 1
    alt = 2 * alt / h0 - 1
    return torch.clip(torch.stack([lat, lon, alt], dim=-1).to(dtype), -1, 1)


class RefNeRFPipeline:
    """nerf.py:16-240 with configs/nerf.json (N_c 64, N_f 128, L_x [14,14,10], L_d 4)."""

    def __init__(self, prep: dict, scale: float, n_bands=4, hidden=256, N_c=64, N_f=128,
                 L_x=(14, 14, 10), L_d=4, lr=5e-4):
        self.prep, self.scale = prep, scale
        self.N_c, self.N_f, self.L_x, self.L_d = N_c, N_f, list(L_x), L_d
        pos, dirc = sum(L_x) * 2, L_d * 6
        self.nerf = {"coarse": RefAtmoNeRF(pos, dirc, n_bands, 1, hidden),
                     "fine": RefAtmoNeRF(pos, dirc, n_bands, n_bands, hidden)}
        params = list(self.nerf["coarse"].parameters()) + list(self.nerf["fine"].parameters())
        self.opt = torch.optim.Adam(params, lr=lr)

    def _forward(self, mode, batch, w_c=None, z_c=None):
        B = batch["origin"].shape[0]
        if mode == "coarse":
            N = self.N_c
            pts, z = sample_uniform(batch["origin"], batch["dir"], batch["len"], N)
        else:
            N = self.N_c + self.N_f
            pts, z = sample_pdf(batch["origin"], batch["dir"], w_c, z_c, self.N_f)
        pts = preprocess_torch(pts, **self.prep)
        pe = positional_encoding(pts, self.L_x).view(B * N, -1)
        dirs = batch["dir"][:, None].repeat(1, N, 1)
        de = positional_encoding(dirs, self.L_d).view(B * N, -1)
        color, sigma = self.nerf[mode](torch.cat([pe, de], dim=1))
        color = torch.exp(torch.clamp(color.view(B, N, -1), max=11))
        sigma = F.relu(sigma.view(B, N, -1))
        cm, _, w = render(z * (self.scale / 1000), color, sigma)
        return cm, w, z

    def train_step(self, batch) -> float:
        cm_c, w_c, z_c = self._forward("coarse", batch)
        cm_f, _, _ = self._forward("fine", batch, w_c, z_c)
        idx = batch["irgb_idx"][:, None]
        loss = (F.mse_loss(torch.take_along_dim(cm_c, idx, 1)[:, 0], batch["rad"])
                + F.mse_loss(torch.take_along_dim(cm_f, idx, 1)[:, 0], batch["rad"]))
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.item()
