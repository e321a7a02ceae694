"""Image metrics the reference reports each epoch (datasets/harp2.py:297-335).

The reference calls torchmetrics' ``peak_signal_noise_ratio(dim=(1, 2), reduction="none",
data_range=...)`` and ``structural_similarity_index_measure(reduction="none")`` on
(V, H, W) cubes. torchmetrics is not installed in this image, so both are restated here
from its published definitions; they run as a handful of device-side torch ops once per
epoch (off the hot path). PSNR is the formula itself; SSIM (Gaussian 11x11 window,
sigma 1.5, k1 = 0.01, k2 = 0.03, reflect padding, border cropped, data range from the
inputs when not given) is parity-unpinned against torchmetrics.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def psnr(pred: torch.Tensor, target: torch.Tensor, data_range: float) -> torch.Tensor:
    """Per-image PSNR of (V, H, W) cubes: 10·log10(range² / mean((p - t)², dims 1, 2))."""
    mse = ((pred - target) ** 2).mean(dim=(1, 2))
    return (2.0 * math.log(data_range) - torch.log(mse)) * (10.0 / math.log(10.0))


def _gaussian_window(size: int, sigma: float, dtype, device) -> torch.Tensor:
    d = torch.arange((1 - size) / 2, (1 + size) / 2, 1.0, dtype=dtype, device=device)
    g = torch.exp(-((d / sigma) ** 2) / 2)
    g = g / g.sum()
    return g[:, None] * g[None, :]


def ssim(pred: torch.Tensor, target: torch.Tensor, data_range: float | None = None,
         kernel_size: int = 11, sigma: float = 1.5, k1: float = 0.01,
         k2: float = 0.03) -> torch.Tensor:
    """Per-image SSIM of (V, 1, H, W) batches (torchmetrics' Gaussian SSIM)."""
    if data_range is None:
        data_range = max((pred.max() - pred.min()).item(), (target.max() - target.min()).item())
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    pad = (kernel_size - 1) // 2
    p = F.pad(pred, (pad, pad, pad, pad), mode="reflect")
    t = F.pad(target, (pad, pad, pad, pad), mode="reflect")
    win = _gaussian_window(kernel_size, sigma, pred.dtype, pred.device)[None, None]
    stats = F.conv2d(torch.cat([p, t, p * p, t * t, p * t]), win)
    mu_p, mu_t, e_pp, e_tt, e_pt = stats.split(pred.shape[0])
    s_pp = (e_pp - mu_p * mu_p).clamp(min=0)
    s_tt = (e_tt - mu_t * mu_t).clamp(min=0)
    s_pt = e_pt - mu_p * mu_t
    ssim_map = ((2 * mu_p * mu_t + c1) * (2 * s_pt + c2)) / (
        (mu_p * mu_p + mu_t * mu_t + c1) * (s_pp + s_tt + c2))
    ssim_map = ssim_map[..., pad:-pad, pad:-pad]
    return ssim_map.reshape(pred.shape[0], -1).mean(-1)


def image_metrics(pred_img: torch.Tensor, target_img: torch.Tensor, max_i: float) -> dict:
    """harp2.py:297-335: max-normalise, clip the prediction to [0, 1], PSNR and SSIM per
    view plus their nan-means."""
    pred = torch.clip(pred_img / max_i, 0, 1)
    target = target_img / max_i
    data_range = (target.max() - target.min()).item()
    p = psnr(pred, target, data_range)
    s = ssim(pred[:, None], target[:, None])
    return {
        "PSNR": p.cpu().tolist(),
        "SSIM": s.cpu().tolist(),
        "PSNR_mean": p[~torch.isnan(p)].mean().item(),
        "SSIM_mean": s[~torch.isnan(s)].mean().item(),
    }
