"""AtmoNeRF — the NeRF MLP of src/atmonr/models/nerf.py:6-144 (same layers, init, skip
connection and noise), f32.

The layers are plain dense GEMMs (M = rays·samples rows, K, N <= 332), run by the ROCm
BLAS libraries through torch.nn.Linear — the library-GEMM case of the design rules; the
NeRF path's custom kernels are the encoder, the pdf sampler, the preprocessor and the
composite. ``forward`` / ``forward_pos_only`` take an optional ``noise`` tensor that
replaces the training-mode ``torch.randn`` draw (parity tests).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn


class AtmoNeRF(nn.Module):
    def __init__(self, pos_channels: int, dir_channels: int, out_channels: int,
                 volume_channels: int, hidden_dim: int = 256) -> None:
        super().__init__()
        self.pos_channels = pos_channels
        self.dir_channels = dir_channels
        self.out_channels = out_channels
        self.volume_channels = volume_channels
        self.hidden_dim = h = hidden_dim
        self.fc1 = nn.Linear(pos_channels, h)
        self.fc2 = nn.Linear(h, h)
        self.fc3 = nn.Linear(h, h)
        self.fc4 = nn.Linear(h, h)
        self.fc5 = nn.Linear(h, h)
        self.fc6 = nn.Linear(h + pos_channels, h)
        self.fc7 = nn.Linear(h, h)
        self.fc8 = nn.Linear(h, h)
        self.fc9 = nn.Linear(h, h + volume_channels)
        self.fc10 = nn.Linear(h + dir_channels, h // 2)
        self.fc11 = nn.Linear(h // 2, out_channels)
        for i in range(1, 12):  # models/nerf.py:45-46
            nn.init.kaiming_normal_(getattr(self, f"fc{i}").weight, mode="fan_out")

    def forward_pos_only(self, x_pos: torch.Tensor, noise: torch.Tensor | None = None):
        """models/nerf.py:48-71: returns (fc9 output, relu(sigma [+ noise if training]))."""
        x = F.relu(self.fc1(x_pos))
        x = F.relu(self.fc2(x))
        x = F.relu(self.fc3(x))
        x = F.relu(self.fc4(x))
        x = F.relu(self.fc5(x))
        x = torch.cat([x, x_pos], dim=1)  # skip connection
        x = F.relu(self.fc6(x))
        x = F.relu(self.fc7(x))
        x = F.relu(self.fc8(x))
        x = self.fc9(x)
        sigma = x[:, self.hidden_dim:]
        if self.training:
            sigma = sigma + (noise if noise is not None
                             else torch.randn(sigma.shape, device=sigma.device))
        return x, F.relu(sigma)

    def forward(self, x: torch.Tensor, noise: torch.Tensor | None = None):
        """models/nerf.py:73-93: (sigmoid color, sigma). fc9's hidden part feeds fc10
        without an activation, as in the reference."""
        x_pos, d = x[:, : self.pos_channels], x[:, self.pos_channels:]
        x, sigma = self.forward_pos_only(x_pos, noise)
        x = F.relu(self.fc10(torch.cat([x[:, : self.hidden_dim], d], dim=1)))
        return torch.sigmoid(self.fc11(x)), sigma


def get_model(hidden_dim: int, N_lambda: int, L_x, L_d: int, include_height: bool
              ) -> tuple[AtmoNeRF, AtmoNeRF]:
    """models/nerf.py:96-144: coarse (1 density) and fine (N_lambda densities) models."""
    if isinstance(L_x, int):
        pos_channels = L_x * 6 + (L_x * 2 if include_height else 0)
    else:
        assert len(L_x) == (4 if include_height else 3)
        pos_channels = sum(L_x) * 2
    dir_channels = L_d * 6
    return (AtmoNeRF(pos_channels, dir_channels, N_lambda, 1, hidden_dim),
            AtmoNeRF(pos_channels, dir_channels, N_lambda, N_lambda, hidden_dim))
