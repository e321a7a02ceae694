"""Volume rendering — same API as src/atmonr/graphics_utils.py:6-77, on the K8 kernels.

``render(z_vals, color, sigma)`` and ``render_with_surface(z_vals, color, sigma,
color_surf)`` return exactly the reference's tuples. Both are differentiable w.r.t.
color, sigma, color_surf and z_vals (the NeRF fine pass back-propagates into z through
sample_pdf). Arithmetic is f32 inside the kernel for any storage dtype; the outputs
have ``color.dtype`` as in the reference (graphics_utils.py:28).
"""

from __future__ import annotations

import torch

from . import _lib
from ._lib import ANRError, call, dtype_code, ptr


class _CompositeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, color, sigma, color_surf, z_scale: float, want_alpha: bool):
        B, N, C = color.shape
        S = sigma.shape[2]
        dt = color.dtype
        dev = color.device
        sigma = sigma.to(dt).contiguous()
        color = color.contiguous()
        cs = color_surf.to(dt).contiguous() if color_surf is not None else None
        zc = z.float().contiguous()
        color_map = torch.empty(B, C, device=dev, dtype=dt)
        atmo = torch.empty(B, C, device=dev, dtype=dt) if cs is not None else None
        surf = torch.empty(B, C, device=dev, dtype=dt) if cs is not None else None
        weights = torch.empty(B, N, S, device=dev, dtype=dt)
        alpha = torch.empty(B, N, S, device=dev, dtype=dt)
        call("anr_composite_fwd", ptr(zc), float(z_scale), ptr(color), ptr(sigma), ptr(cs),
             dtype_code(dt), B, N, C, S, ptr(color_map), ptr(atmo), ptr(surf), ptr(weights),
             ptr(alpha), _lib.stream(dev))
        ctx.save_for_backward(zc, color, sigma, cs)
        # outputs the loss does not use (alpha, weights, atmo, surf in training) arrive as
        # None instead of materialised zero tensors: the kernel skips null gradients
        ctx.set_materialize_grads(False)
        ctx.z_scale = float(z_scale)
        ctx.has_surf = cs is not None
        ctx.z_dtype = z.dtype
        if cs is None:
            return color_map, alpha, weights
        return color_map, alpha, weights, atmo, surf

    @staticmethod
    def backward(ctx, *grads):
        zc, color, sigma, cs = ctx.saved_tensors
        B, N, C = color.shape
        S = sigma.shape[2]
        dt = color.dtype
        dev = color.device
        if ctx.has_surf:
            g_cm, g_alpha, g_w, g_atmo, g_surf = grads
        else:
            g_cm, g_alpha, g_w = grads
            g_atmo = g_surf = None

        def prep(g):
            return None if g is None else g.to(dt).contiguous()

        if g_cm is None:  # the kernel requires dL/dcolor_map
            g_cm = torch.zeros(B, color.shape[2], device=dev, dtype=dt)

        need_z, need_c, need_s, need_cs = ctx.needs_input_grad[:4]
        d_color = torch.empty_like(color) if need_c else None
        d_sigma = torch.empty_like(sigma) if need_s else None
        d_cs = torch.empty_like(cs) if (need_cs and cs is not None) else None
        d_z = torch.empty(B, N, device=dev, dtype=torch.float32) if need_z else None
        call("anr_composite_bwd", ptr(zc), ctx.z_scale, ptr(color), ptr(sigma), ptr(cs),
             dtype_code(dt), B, N, C, S, ptr(prep(g_cm)), ptr(prep(g_atmo)),
             ptr(prep(g_surf)), ptr(prep(g_w)), ptr(prep(g_alpha)), ptr(d_color),
             ptr(d_sigma), ptr(d_cs), ptr(d_z), _lib.stream(dev))
        if d_z is not None:
            d_z = d_z.to(ctx.z_dtype)
        return d_z, d_color, d_sigma, d_cs, None, None


def _check(z_vals, color, sigma):
    if not (z_vals.dim() == 2 and color.dim() == 3 and sigma.dim() == 3):
        raise ANRError("render: expected z (B,N), color (B,N,C), sigma (B,N,S)")
    if z_vals.shape != color.shape[:2] or z_vals.shape != sigma.shape[:2]:
        raise ANRError("render: z / color / sigma shapes disagree")
    if color.dtype not in (torch.float16, torch.float32):
        raise ANRError(f"render: unsupported dtype {color.dtype}")


def render(z_vals: torch.Tensor, color: torch.Tensor, sigma: torch.Tensor, z_scale: float = 1.0):
    """graphics_utils.py:6-49. Returns (color_map, alpha, weights).

    ``z_scale`` multiplies z in f32 inside the kernel (the pipelines pass scale/1000
    here instead of materialising z_vals*(scale/1000), instant_ngp.py:188).
    """
    _check(z_vals, color, sigma)
    return _CompositeFn.apply(z_vals, color, sigma, None, z_scale, True)


def render_with_surface(z_vals, color, sigma, color_surf, z_scale: float = 1.0):
    """graphics_utils.py:52-77. Returns (color_map, alpha, weights, atmo, surf)."""
    _check(z_vals, color, sigma)
    return _CompositeFn.apply(z_vals, color, sigma, color_surf, z_scale, True)
