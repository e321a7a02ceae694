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


class _PreprocessFn(torch.autograd.Function):
    """harp2.py:372-386 on the GPU (K2); differentiable w.r.t. the points — the NeRF
    pipeline back-propagates through it into the pdf samples."""

    @staticmethod
    def forward(ctx, flat, prep):
        out = torch.empty_like(flat)
        call("anr_preprocess_points", ptr(flat), flat.shape[0], prep, ptr(out),
             _lib.stream(flat.device))
        ctx.save_for_backward(flat)
        ctx.prep = prep
        return out

    @staticmethod
    def backward(ctx, d_out):
        (flat,) = ctx.saved_tensors
        d_out = d_out.float().contiguous()
        d_in = torch.empty_like(flat)
        call("anr_preprocess_points_bwd", ptr(flat), flat.shape[0], ctx.prep, ptr(d_out),
             ptr(d_in), _lib.stream(flat.device))
        return d_in, None


def preprocess_points(pts: torch.Tensor, prep: "_lib.PrepParams") -> torch.Tensor:
    """Apply a preprocessor to arbitrary points (..., 3); differentiable w.r.t. f32 pts.

    f64 points (the extract path, scripts/extract.py:206) are preprocessed in f64 end to
    end and returned as f32 coordinates (what the hash encoder consumes); no gradient."""
    shp = pts.shape
    if pts.dtype == torch.float64:
        if pts.requires_grad:
            raise _lib.ANRError("preprocess_points: f64 points are inference-only")
        flat = pts.reshape(-1, 3).contiguous()
        out = torch.empty(flat.shape, device=flat.device, dtype=torch.float32)
        call("anr_preprocess_points_f64", ptr(flat), flat.shape[0], prep, ptr(out),
             _lib.stream(flat.device))
        return out.view(shp)
    flat = pts.reshape(-1, 3).float().contiguous()
    return _PreprocessFn.apply(flat, prep).view(shp)


class _SamplePdfFn(torch.autograd.Function):
    """samplers.py:50-103: one wavefront per ray (searchsorted on an f64-accumulated cdf,
    rank sort of coarse + fine z); backward into the coarse weights through t_in_bin."""

    @staticmethod
    def forward(ctx, weights, z_c, u, origin, direction, n_samples):
        B, Nc = z_c.shape
        dev = z_c.device
        Nt = Nc + n_samples
        w = weights.float().contiguous()
        z = torch.empty(B, Nt, device=dev)
        pts = torch.empty(B, Nt, 3, device=dev)
        src = torch.empty(B, Nt, device=dev, dtype=torch.int32)
        inds = torch.empty(B, n_samples, device=dev, dtype=torch.int32)
        cdf = torch.empty(B, Nc - 1, device=dev)
        call("anr_sample_pdf_fwd", ptr(w), w.stride(0), w.stride(1), ptr(z_c), ptr(u),
             ptr(origin), ptr(direction), B, Nc, n_samples, ptr(z), ptr(pts), ptr(src),
             ptr(inds), ptr(cdf), _lib.stream(dev))
        ctx.save_for_backward(w, z_c, u, direction, src, inds, cdf)
        ctx.n_samples = n_samples
        return pts, z

    @staticmethod
    def backward(ctx, d_pts, d_z):
        w, z_c, u, direction, src, inds, cdf = ctx.saved_tensors
        B, Nc = z_c.shape
        d_w = torch.zeros_like(w)
        d_pts = d_pts.float().contiguous() if d_pts is not None else None
        d_z = d_z.float().contiguous() if d_z is not None else None
        call("anr_sample_pdf_bwd", ptr(w), w.stride(0), w.stride(1), ptr(z_c), ptr(u),
             ptr(direction), ptr(src), ptr(inds), ptr(cdf), B, Nc, ctx.n_samples, ptr(d_z),
             ptr(d_pts), ptr(d_w), _lib.stream(w.device))
        return d_w, None, None, None, None, None


def sample_pdf(ray_batch: Mapping[str, torch.Tensor], pdf_discrete: torch.Tensor,
               z_vals_c: torch.Tensor, n_samples: int = 128, u: torch.Tensor | None = None
               ) -> tuple[torch.Tensor, torch.Tensor]:
    """samplers.py:50-103. pdf_discrete (B, Nc, S) — channel 0 is the pdf (the render
    weights); u (B, n_samples) overrides the torch.rand draws. Returns pts (B, Nc+n, 3) and
    sorted z (B, Nc+n); gradients reach pdf_discrete as in the reference."""
    origin = ray_batch["origin"].float().contiguous()
    direction = ray_batch["dir"].float().contiguous()
    B, Nc = z_vals_c.shape
    if u is None:
        u = torch.rand(B, n_samples, device=z_vals_c.device)
    u = u.float().contiguous()
    return _SamplePdfFn.apply(pdf_discrete, z_vals_c.float().contiguous(), u, origin,
                              direction, n_samples)
