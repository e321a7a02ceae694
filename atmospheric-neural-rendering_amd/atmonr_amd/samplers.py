"""Ray samplers — same API as src/atmonr/samplers.py, computed by libanr_hip.so.

``sample_uniform_bins`` (samplers.py:8-47) runs the K1 kernel: identical z and pts to
the reference for identical uniform draws (the draws come from ``torch.rand`` with the
same shape, so a seeded run reproduces the reference's samples). The kernel can also
apply the HARP2 "horizontal" point preprocessor and the Instant-NGP remap in the same
pass (:func:`sample_and_preprocess`), which the pipelines use.
"""

from __future__ import annotations

from typing import Mapping

import torch

from . import _lib
from ._lib import call, ptr

_BINS: dict[tuple[int, torch.device], torch.Tensor] = {}


def _bins(n_bins: int, device: torch.device) -> torch.Tensor:
    key = (n_bins, device)
    if key not in _BINS:
        # torch.linspace(0, 1, n+1) exactly as samplers.py:34 builds it
        _BINS[key] = torch.linspace(0, 1, n_bins + 1, device=device)
    return _BINS[key]


def _uniform(B: int, n_bins: int, device, random: bool, generator=None):
    if not random:
        return None
    return torch.rand((B, n_bins), device=device, generator=generator)


def sample_uniform_bins(
    ray_batch: Mapping[str, torch.Tensor],
    n_bins: int = 64,
    random: bool = True,
    u: torch.Tensor | None = None,
) -> tuple[torch.Tensor, torch.Tensor]:
    """Stratified samples along each ray (samplers.py:8-47).

    Returns pts (B, n_bins, 3) and z_vals (B, n_bins). ``u`` overrides the uniform
    draws (B, n_bins) (used by parity tests); otherwise they come from torch.rand as in
    the reference.
    """
    origin, direction, length = ray_batch["origin"], ray_batch["dir"], ray_batch["len"]
    B = origin.shape[0]
    device = origin.device
    if u is None:
        u = _uniform(B, n_bins, device, random)
    if u is not None:  # bound to a name: a temporary's block could be reused by _bins()
        u = u.float().contiguous()
    origin = origin.float().contiguous()
    direction = direction.float().contiguous()
    length = length.float().contiguous()
    pts = torch.empty(B, n_bins, 3, device=device)
    z = torch.empty(B, n_bins, device=device)
    call("anr_sample_uniform_bins", ptr(origin), ptr(direction), ptr(length),
         ptr(u), ptr(_bins(n_bins, device)), B, n_bins,
         ptr(pts), ptr(z), None, None, _lib.stream(device))
    return pts, z


def sample_and_preprocess(
    ray_batch: Mapping[str, torch.Tensor],
    n_bins: int,
    prep: "_lib.PrepParams",
    random: bool = True,
    u: torch.Tensor | None = None,
    want_pts: bool = False,
) -> tuple[torch.Tensor | None, torch.Tensor, torch.Tensor]:
    """Fused K1+K2: samples, z and the preprocessed (+remapped) hash-grid coordinates.

    Returns (pts or None, z (B, n_bins), coords (B, n_bins, 3)).
    """
    origin, direction, length = ray_batch["origin"], ray_batch["dir"], ray_batch["len"]
    B = origin.shape[0]
    device = origin.device
    if u is None:
        u = _uniform(B, n_bins, device, random)
    if u is not None:  # bound to a name: a temporary's block could be reused by _bins()
        u = u.float().contiguous()
    origin = origin.float().contiguous()
    direction = direction.float().contiguous()
    length = length.float().contiguous()
    pts = torch.empty(B, n_bins, 3, device=device) if want_pts else None
    z = torch.empty(B, n_bins, device=device)
    coords = torch.empty(B, n_bins, 3, device=device)
    call("anr_sample_uniform_bins", ptr(origin), ptr(direction), ptr(length),
         ptr(u), ptr(_bins(n_bins, device)), B, n_bins,
         ptr(pts), ptr(z), prep, ptr(coords), _lib.stream(device))
    return pts, z, coords


def preprocess_points(pts: torch.Tensor, prep: "_lib.PrepParams") -> torch.Tensor:
    """Apply a preprocessor to arbitrary points (..., 3) (extract path)."""
    shp = pts.shape
    flat = pts.reshape(-1, 3).float().contiguous()
    out = torch.empty_like(flat)
    call("anr_preprocess_points", ptr(flat), flat.shape[0], prep, ptr(out),
         _lib.stream(pts.device))
    return out.view(shp)
