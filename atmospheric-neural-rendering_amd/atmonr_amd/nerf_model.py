"""AtmoNeRF — the NeRF MLP of src/atmonr/models/nerf.py:6-144 (same layers, init, skip
connection and noise), f32.

The layers are plain dense GEMMs (M = rays·samples rows, K, N <= 332), run by the ROCm
BLAS libraries through torch.nn.Linear — the library-GEMM case of the design rules; the
NeRF path's custom kernels are the encoder, the pdf sampler, the preprocessor and the
composite. ``forward`` / ``forward_pos_only`` take an optional ``noise`` tensor that
replaces the training-mode ``torch.randn`` draw (parity tests).
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn


def _column_sum(g: torch.Tensor) -> torch.Tensor:
    """g.sum(0) for a tall (M, C) gradient in two stages: torch's one-pass column
    reduction runs a handful of blocks when C is not a multiple of 4 (fc9's 257 / 260
    outputs: 3.9 ms per step at 786 K rows); 512 row groups first spread it over the chip."""
    M, C = g.shape
    S = 512
    if M < 64 * S:
        return g.sum(0)
    r = M // S
    out = g[: S * r].view(S, r, C).sum(1).sum(0)
    if S * r < M:
        out = out + g[S * r:].sum(0)
    return out


# split of the weight-gradient GEMMs (bench sweep, S = 1/8/16/32/64/128:
# 61.1/52.7/47.1/45.1/43.6/50.0 ms per NeRF step)
_SPLIT_K = int(os.environ.get("ANR_NERF_SPLITK", "64"))


def _weight_grad(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """g^T x for the tall (M rows) operands of a layer's weight gradient. As one GEMM the
    (out x in) result has only 32 tiles to spread over 256 CUs; split over the M rows into
    a batched GEMM of _SPLIT_K slices (bmm), then summed — same products, f32 partial sums
    added in a different order."""
    M = g.shape[0]
    S = _SPLIT_K
    if S <= 1 or M < S * 4096 or M % S:
        return g.t() @ x
    r = M // S
    return torch.bmm(g.view(S, r, g.shape[1]).transpose(1, 2), x.view(S, r, x.shape[1])).sum(0)


class _LinearFn(torch.autograd.Function):
    """F.linear with the same backward GEMMs as autograd's, but the bias gradient by
    _column_sum (summation order differs from autograd's by f32 rounding only)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        g = g.contiguous()
        dx = g @ weight if ctx.needs_input_grad[0] else None
        dw = _weight_grad(g, x) if ctx.needs_input_grad[1] else None
        db = _column_sum(g) if ctx.needs_input_grad[2] else None
        return dx, dw, db


class _LinearReLUFn(torch.autograd.Function):
    """relu(F.linear(x, W, b)) as one library GEMM with a bias + ReLU epilogue
    (torch._addmm_activation, which has no autograd formula) and the matching backward:
    g' = g where y > 0 (relu's subgradient at 0 is 0, as torch's), then the GEMMs."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        y = torch._addmm_activation(bias, x, weight.t())
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, y = ctx.saved_tensors
        g = g.contiguous()
        M, C = g.shape
        if C % 4 == 0 and C <= 1024 and y.is_contiguous() and M >= 256:
            # one pass: mask + per-block column sums (anr_relu_bwd_colsum)
            from . import _lib

            parts = min(1024, M // 256)
            gm = torch.empty_like(g)
            partial = torch.empty(parts, C, device=g.device, dtype=torch.float32)
            _lib.call("anr_relu_bwd_colsum", _lib.ptr(g), _lib.ptr(y), M, C, _lib.ptr(gm),
                      _lib.ptr(partial), parts, _lib.stream(g.device))
            db = partial.sum(0) if ctx.needs_input_grad[2] else None
        else:
            gm = torch.ops.aten.threshold_backward(g, y, 0)
            db = _column_sum(gm) if ctx.needs_input_grad[2] else None
        dx = gm @ weight if ctx.needs_input_grad[0] else None
        dw = _weight_grad(gm, x) if ctx.needs_input_grad[1] else None
        return dx, dw, db


def _linear_relu(layer: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32:
        if torch.is_grad_enabled():
            return _LinearReLUFn.apply(x, layer.weight, layer.bias)
        return torch._addmm_activation(layer.bias, x, layer.weight.t())
    return F.relu(layer(x))


class _Linear(nn.Linear):
    """nn.Linear (same parameters and state-dict keys) with _LinearFn's backward: split-K
    weight gradient, and a bias gradient that avoids torch's slow narrow-column reduction
    (out_features not a multiple of 4)."""

    def forward(self, x):
        if torch.is_grad_enabled() and x.is_cuda and x.dim() == 2:
            return _LinearFn.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)


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
        self.fc9 = _Linear(h, h + volume_channels)
        self.fc10 = nn.Linear(h + dir_channels, h // 2)
        self.fc11 = _Linear(h // 2, out_channels)
        for i in range(1, 12):  # models/nerf.py:45-46
            nn.init.kaiming_normal_(getattr(self, f"fc{i}").weight, mode="fan_out")

    def forward_pos_only(self, x_pos: torch.Tensor, noise: torch.Tensor | None = None):
        """models/nerf.py:48-71: returns (fc9 output, relu(sigma [+ noise if training]))."""
        x = _linear_relu(self.fc1, x_pos)
        x = _linear_relu(self.fc2, x)
        x = _linear_relu(self.fc3, x)
        x = _linear_relu(self.fc4, x)
        x = _linear_relu(self.fc5, x)
        x = torch.cat([x, x_pos], dim=1)  # skip connection
        x = _linear_relu(self.fc6, x)
        x = _linear_relu(self.fc7, x)
        x = _linear_relu(self.fc8, x)
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
        x = _linear_relu(self.fc10, torch.cat([x[:, : self.hidden_dim], d], dim=1))
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
