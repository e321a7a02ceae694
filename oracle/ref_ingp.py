"""ORACLE (test infrastructure only): the Instant-NGP train step on CPU, with autograd.

Restates src/atmonr/pipelines/instant_ngp.py:137-206 (forward) and :249-263
(compute_loss) in float64 torch on top of the other oracle pieces:

* sampler            samplers.py:8-47             -> ref_path.sample_uniform_bins
* point preprocessor harp2.py:357-388             -> ref_nerf.preprocess_torch
* remap              instant_ngp.py:143-160       -> (p + 1) / 2, z / alt_compress_factor
* tcnn HashGrid      instant_ngp.py:60-63,163     -> hashgrid() below, corners and weights
                                                     from ref_tcnn.hashgrid_corners
* tcnn FullyFusedMLP instant_ngp.py:64-77,164-171 -> ref_tcnn.mlp_fwd
* SH2 + Identity     instant_ngp.py:69-72,165-169 -> ref_tcnn.sh + the pos_out columns
* surface path       instant_ngp.py:78-85,173-174
* composite          graphics_utils.py:52-77      -> ref_path.render_with_surface
* loss               instant_ngp.py:249-263       -> ref_path.LOSSES
* AdamW groups       instant_ngp.py:107-127

``half=True`` rounds what the f16 GPU path rounds (hash table, encodings, MLP weights
and hidden activations, the f16 MLP outputs) so the oracle tracks the bench
configuration; gradients pass through the roundings unchanged (casts are identity in
autograd). tcnn semantics are unpinned against real tinycudann (see ref_tcnn).
"""

from __future__ import annotations

import numpy as np
import torch

from . import ref_nerf, ref_path, ref_tcnn

MODULES = ("pos_encoder", "pos_mlp", "dir_mlp", "surf_encoder", "surf_mlp")


def _grid_cfg(enc_cfg: dict, n_dims: int):
    return (n_dims, int(enc_cfg["n_levels"]), int(enc_cfg["base_resolution"]),
            float(enc_cfg["per_level_scale"]), int(enc_cfg["log2_hashmap_size"]))


def hashgrid(x: torch.Tensor, table: torch.Tensor, cfg, rnd) -> torch.Tensor:
    """tcnn GridEncoding forward, differentiable in ``table``; x (M, D) float32."""
    xn = x.detach().float().numpy()
    tab = rnd(table).view(-1, 2)
    outs = []
    for lvl in range(cfg[1]):
        idx, wt = ref_tcnn.hashgrid_corners(xn, cfg, lvl)
        outs.append(torch.einsum("mc,mcf->mf", torch.from_numpy(wt),
                                 tab[torch.from_numpy(idx)]))
    return rnd(torch.cat(outs, dim=1))


class RefInstantNGP:
    """Parameters (float64 leaf tensors, flat per module like tcnn) + forward / loss."""

    def __init__(self, config: dict, state: dict, prep: dict, scale: float, max_i: float,
                 half: bool = False, mlp_half=None):
        self.cfg = config
        self.ingp = config["instant_ngp"]
        self.N = int(config["num_samples_per_ray"])
        self.nb = int(config["num_bands"])
        self.alt = float(config["alt_compress_factor"])
        self.prep, self.scale, self.max_i = prep, float(scale), float(max_i)
        self.half = half
        # rounding of the per-sample pos / dir MLPs: as the rest (None) or "bf16" (the
        # build's bf16 MFMA field, BASELINE configs[4])
        self.mlp_half = half if mlp_half is None else mlp_half
        self.params = {m: state[m]["params"].detach().cpu().double().clone().requires_grad_(True)
                       for m in MODULES}
        self.pos_grid = _grid_cfg(self.ingp["encoding"], 3)
        self.surf_grid = _grid_cfg(self.ingp["surface_encoding"]["nested"][0], 2)

    def _rnd(self, t):
        return t.half().double() if self.half else t

    def _mlp(self, x, p, n_in, n_out, net_cfg, half=None):
        half = self.half if half is None else half
        y = ref_tcnn.mlp_fwd(x, p, n_in, n_out, int(net_cfg["n_neurons"]),
                             int(net_cfg["n_hidden_layers"]), half=half)
        return ref_tcnn.rounder(half)(y)

    def forward(self, b: dict, u: torch.Tensor | None) -> dict:
        """instant_ngp.py:137-206 on a CPU ray batch; u (B, N) or None (bin midpoints)."""
        P = self.params
        B, N = b["origin"].shape[0], self.N
        pts, z = ref_path.sample_uniform_bins(b["origin"], b["dir"], b["len"], u=u, n_bins=N)
        pts = ref_nerf.preprocess_torch(pts, **self.prep)
        pts = (pts + 1) / 2
        pts = torch.cat([pts[..., :2], pts[..., 2:] / self.alt], dim=-1)
        pos_enc = hashgrid(pts.reshape(B * N, 3), P["pos_encoder"], self.pos_grid, self._rnd)
        pos_out = self._mlp(pos_enc, P["pos_mlp"], 32, 16, self.ingp["network"],
                            self.mlp_half)
        dirs = b["dir"][:, None].expand(B, N, 3).reshape(B * N, 3)
        sh = torch.from_numpy(ref_tcnn.sh(dirs.numpy(), 2))
        dir_enc = torch.cat([self._rnd(sh), pos_out[:, 1:]], dim=1)  # SH2 | Identity (19)
        color = torch.relu(self._mlp(dir_enc, P["dir_mlp"], 19, self.nb,
                                     self.ingp["rgb_network"], self.mlp_half))
        sigma = torch.relu(pos_out[:, :1])
        # surface (instant_ngp.py:143,150,173-174): normalized Cartesian x, y
        ps = (b["origin"] + b["dir"] * b["len"][:, None] + 1) / 2
        surf_sh = self._rnd(torch.from_numpy(ref_tcnn.sh(b["dir"].numpy(), 2)))
        surf_enc = torch.cat([hashgrid(ps[:, :2], P["surf_encoder"], self.surf_grid,
                                       self._rnd), surf_sh], dim=1)
        color_surf = torch.relu(self._mlp(surf_enc, P["surf_mlp"], 36, self.nb,
                                          self.ingp["surface_network"]))
        # the composite in f32, as the reference evaluates graphics_utils.py in the network
        # output dtype (alpha = 1 - exp(-sigma * delta) cancels in that precision; the
        # GPU composite computes in f32 for every storage dtype)
        cm, alpha, weights, atmo, surf = ref_path.render_with_surface(
            z * (self.scale / 1000), color.view(B, N, -1).float(),
            sigma.view(B, N, 1).float(), color_surf.float())
        return {"color_map_fine": cm.double(), "color_map_atmo": atmo.double(),
                "color_map_surf": surf.double(), "weights_fine": weights, "z_vals_fine": z,
                "color_fine": color.view(B, N, -1)[:, :-1],
                "sigma_fine": sigma.view(B, N, 1)[:, :-1], "color_surf": color_surf}

    def loss(self, b: dict, res: dict, name: str = "mse_plus_hdr") -> torch.Tensor:
        """instant_ngp.py:249-263: loss_fn(take_along_dim(color_map, irgb), rad, max_i)."""
        pred = torch.take_along_dim(res["color_map_fine"], b["irgb_idx"][:, None], 1)[:, 0]
        return ref_path.LOSSES[name](pred, b["rad"].double(), self.max_i)

    def optimizer(self, opt_cfg: dict) -> torch.optim.Optimizer:
        """AdamW, weight decay on the MLPs only (instant_ngp.py:107-127)."""
        groups = [{"params": [self.params[m] for m in ("pos_encoder", "surf_encoder")],
                   "weight_decay": 0.0},
                  {"params": [self.params[m] for m in ("pos_mlp", "dir_mlp", "surf_mlp")],
                   "weight_decay": opt_cfg["weight_decay"]}]
        return torch.optim.AdamW(groups, lr=opt_cfg["lr"], betas=tuple(opt_cfg["betas"]),
                                 eps=opt_cfg["eps"])


def cpu_batch(b: dict) -> dict:
    return {k: v.detach().cpu() for k, v in b.items()}


def prep_kwargs(pp) -> dict:
    """Constants of a dataset's horizontal point preprocessor (harp2.py:357-370)."""
    return dict(scale=float(pp.scale),
                offset=torch.tensor(np.asarray(pp.offset, dtype=np.float64)),
                lat_min=pp.lat_min, lat_range=pp.lat_range, lon_min=pp.lon_min,
                lon_range=pp.lon_range, h0=pp.ray_origin_height, shift_lon=pp.shift_lon)
