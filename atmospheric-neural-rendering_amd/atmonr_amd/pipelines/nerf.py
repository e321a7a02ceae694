"""NeRFPipeline — src/atmonr/pipelines/nerf.py:16-273 on the MI355X path.

Per stage (coarse: N_c stratified samples; fine: N_c + N_f from the coarse weights):
    sampler (K1, or the pdf sampler)  -> preprocessor (K2, differentiable)
    -> positional encoding of points and directions into one (B·N, 100) buffer
    -> AtmoNeRF (f32 library GEMMs) -> exp(clamp(color, 11)), relu(sigma)
    -> composite (K8, plain render)
Gradients reach the coarse network through the fine samples (sample_pdf's t_in_bin ->
preprocessor -> encoding), as in the reference. The loss is the sum of the coarse and
fine MSEs (nerf.py:219-240); the optimizer is Adam (nerf.py:56-71) run by FusedAdam.

``forward(ray_batch, u_coarse=None, u_fine=None, noise=None)``: optional overrides of the
uniform draws and of the training-mode density noise (dict "coarse"/"fine"), used by the
parity tests; without them the draws come from torch.rand / torch.randn as in the
reference.
"""

from __future__ import annotations

from itertools import chain
from typing import Any, Mapping

import torch
import torch.nn.functional as F
from torch.optim import Optimizer

from ..encoders import nerf_input, positional_encoding
from ..graphics_utils import render
from ..nerf_model import get_model
from ..optim import FusedAdam
from ..samplers import preprocess_points, sample_pdf, sample_uniform_bins
from .pipeline import Pipeline


class NeRFPipeline(Pipeline):
    def __init__(self, config: dict, dataset: Any) -> None:
        super().__init__(config, dataset)
        if config["include_height"]:
            raise NotImplementedError("include_height is disabled in both reference configs")
        self.nerf = {}
        self.nerf["coarse"], self.nerf["fine"] = get_model(
            hidden_dim=config["mlp_hidden_dim"], N_lambda=config["num_bands"],
            L_x=config["encoder"]["L_x"], L_d=config["encoder"]["L_d"],
            include_height=config["include_height"])
        self.training = True
        self._prep = (self.point_preprocessor.params()
                      if self.point_preprocessor is not None else None)

    def send_tensors_to(self, device: int) -> None:
        self.device = device
        self.nerf["coarse"] = self.nerf["coarse"].to(device)
        self.nerf["fine"] = self.nerf["fine"].to(device)

    def parameters(self):
        return chain(self.nerf["coarse"].parameters(), self.nerf["fine"].parameters())

    def get_optimizer(self, config: dict, fused: bool = True) -> Optimizer:
        """nerf.py:56-71: Adam over both networks."""
        if fused:
            return FusedAdam(self.parameters(), lr=config["lr"], decoupled=False)
        return torch.optim.Adam(self.parameters(), lr=config["lr"])

    def _forward(self, mode: str, ray_batch: Mapping[str, torch.Tensor],
                 weights_coarse: torch.Tensor | None = None,
                 z_vals_coarse: torch.Tensor | None = None,
                 u: torch.Tensor | None = None, noise: torch.Tensor | None = None
                 ) -> dict[str, torch.Tensor]:
        """nerf.py:73-177."""
        assert (mode == "coarse" and z_vals_coarse is None) or (
            mode == "fine" and z_vals_coarse is not None)
        B_ = ray_batch["origin"].shape[0]
        if mode == "coarse":
            N = self.config["sampler"]["N_c"]
            pts, z_vals = sample_uniform_bins(ray_batch, n_bins=N, u=u)
        else:
            N = self.config["sampler"]["N_c"] + self.config["sampler"]["N_f"]
            pts, z_vals = sample_pdf(ray_batch, weights_coarse, z_vals_coarse,
                                     n_samples=self.config["sampler"]["N_f"], u=u)
        if self._prep is not None:
            pts = preprocess_points(pts, self._prep)
        x = nerf_input(pts, ray_batch["dir"], self.config["encoder"]["L_x"],
                       self.config["encoder"]["L_d"])
        color, sigma = self.nerf[mode](x, noise)
        color = color.view(B_, N, -1)
        sigma = sigma.view(B_, N, 1) if mode == "coarse" else sigma.view(B_, N, -1)
        color = torch.exp(torch.clamp(color, max=11))
        sigma = F.relu(sigma)
        color_map, _, weights = render(z_vals, color, sigma, z_scale=self.scale / 1000)
        return {
            f"color_{mode}": color,
            f"sigma_{mode}": sigma,
            f"color_map_{mode}": color_map,
            f"weights_{mode}": weights,
            f"z_vals_{mode}": z_vals,
        }

    def forward(self, ray_batch: Mapping[str, torch.Tensor],
                u_coarse: torch.Tensor | None = None, u_fine: torch.Tensor | None = None,
                noise: Mapping[str, torch.Tensor] | None = None) -> dict[str, torch.Tensor]:
        """nerf.py:179-198."""
        noise = noise or {}
        results = self._forward("coarse", ray_batch, u=u_coarse, noise=noise.get("coarse"))
        results.update(self._forward(
            "fine", ray_batch, weights_coarse=results["weights_coarse"],
            z_vals_coarse=results["z_vals_coarse"], u=u_fine, noise=noise.get("fine")))
        return results

    def extract(self, pts: torch.Tensor) -> torch.Tensor:
        """nerf.py:200-217: fine-model density at normalized scene points (P, 3)."""
        with torch.no_grad():
            if self._prep is not None:
                pts = preprocess_points(pts, self._prep)
            pts_enc = positional_encoding(pts, self.config["encoder"]["L_x"]).view(
                pts.shape[0], -1)
            _, sigma = self.nerf["fine"].forward_pos_only(pts_enc)
        return torch.clip(sigma, min=0)

    def compute_loss(self, ray_batch: Mapping[str, torch.Tensor],
                     results: dict[str, torch.Tensor]) -> torch.Tensor:
        """nerf.py:219-240: mse(coarse) + mse(fine) on the observed band."""
        idx = ray_batch["irgb_idx"][:, None]
        rc = torch.take_along_dim(results["color_map_coarse"], idx, 1)[:, 0]
        rf = torch.take_along_dim(results["color_map_fine"], idx, 1)[:, 0]
        return F.mse_loss(rc, ray_batch["rad"]) + F.mse_loss(rf, ray_batch["rad"])

    def state_dict(self) -> Mapping[str, Mapping[str, Any]]:
        return {"coarse": self.nerf["coarse"].state_dict(),
                "fine": self.nerf["fine"].state_dict()}

    def load_state_dict(self, state_dict: dict) -> None:
        self.nerf["coarse"].load_state_dict(state_dict["coarse"])
        self.nerf["fine"].load_state_dict(state_dict["fine"])

    def train(self) -> None:
        self.training = True
        self.nerf["coarse"].train()
        self.nerf["fine"].train()

    def eval(self) -> None:
        self.training = False
        self.nerf["coarse"].eval()
        self.nerf["fine"].eval()
