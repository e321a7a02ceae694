"""Positional encoding — same API as src/atmonr/encoders.py, computed by libanr_hip.so.

``positional_encoding(pts, L)`` (encoders.py:4-28) returns the reference's shapes: an int
L gives (P, D, 2L) with interleaved (sin, cos) pairs per frequency, a list L gives
(..., 2·ΣL) with per-coordinate [sin…, cos…] blocks. Frequencies are (2^l·π) in f32 times
the coordinate in f32, as the reference computes them. Differentiable w.r.t. the points.

``nerf_input`` builds the NeRF MLP input cat[PE(pts, L_x), PE(dirs, L_d)] (nerf.py:125-
136) in one buffer, reading each ray's direction once per sample instead of materialising
``dirs.repeat(1, N, 1)``.
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, ptr


class _PosencFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, desc, width):
        P = x.shape[0]
        out = torch.empty(P, width, device=x.device)
        call("anr_posenc_fwd", ctypes.byref(desc), ptr(x), 1, P, ptr(out), width,
             _lib.stream(x.device))
        ctx.save_for_backward(x)
        ctx.desc = desc
        return out

    @staticmethod
    def backward(ctx, d_out):
        (x,) = ctx.saved_tensors
        d_out = d_out.float().contiguous()
        dx = torch.empty_like(x)
        call("anr_posenc_bwd", ctypes.byref(ctx.desc), ptr(x), x.shape[0], ptr(d_out),
             d_out.stride(0), ptr(dx), _lib.stream(x.device))
        return dx, None, None


def positional_encoding(pts: torch.Tensor, L: int | list[int]) -> torch.Tensor:
    """encoders.py:4-28 (shapes and column order of the reference)."""
    D = pts.shape[-1]
    desc = _lib.posenc_desc(L, D)
    width = _lib.load().anr_posenc_width(ctypes.byref(desc))
    x = pts.reshape(-1, D).float().contiguous()
    out = _PosencFn.apply(x, desc, width)
    if isinstance(L, int):
        return out.view(x.shape[0], D, 2 * L)
    return out.view(*pts.shape[:-1], width)


class _NerfInputFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pts, dirs, n_per_ray, dx, dd, wx, wd):
        P = pts.shape[0]
        x = torch.empty(P, wx + wd, device=pts.device)
        s = _lib.stream(pts.device)
        call("anr_posenc_fwd", ctypes.byref(dx), ptr(pts), 1, P, ptr(x), wx + wd, s)
        call("anr_posenc_fwd", ctypes.byref(dd), ptr(dirs), n_per_ray, P, ptr(x) + 4 * wx,
             wx + wd, s)
        ctx.save_for_backward(pts)
        ctx.dx, ctx.stride = dx, wx + wd
        return x

    @staticmethod
    def backward(ctx, d_x):
        (pts,) = ctx.saved_tensors
        d_x = d_x.float().contiguous()
        d_pts = torch.empty_like(pts)
        call("anr_posenc_bwd", ctypes.byref(ctx.dx), ptr(pts), pts.shape[0], ptr(d_x),
             ctx.stride, ptr(d_pts), _lib.stream(pts.device))
        return d_pts, None, None, None, None, None, None


def nerf_input(pts: torch.Tensor, dirs: torch.Tensor, L_x, L_d: int) -> torch.Tensor:
    """cat[PE(pts, L_x), PE(dirs repeated per sample, L_d)]: pts (B, N, 3), dirs (B, 3)
    -> (B·N, 2ΣL_x + 6·L_d). Differentiable w.r.t. pts (the directions are data)."""
    B, N = pts.shape[0], pts.shape[1]
    dx, dd = _lib.posenc_desc(L_x, 3), _lib.posenc_desc(L_d, 3)
    lib = _lib.load()
    wx, wd = lib.anr_posenc_width(ctypes.byref(dx)), lib.anr_posenc_width(ctypes.byref(dd))
    return _NerfInputFn.apply(pts.reshape(B * N, 3).float().contiguous(),
                              dirs.float().contiguous(), N, dx, dd, wx, wd)
