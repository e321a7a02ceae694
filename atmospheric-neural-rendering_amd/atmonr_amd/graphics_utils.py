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
        args = (ptr(zc), ctx.z_scale, ptr(color), ptr(sigma), ptr(cs), dtype_code(dt), B, N, C,
                S, ptr(prep(g_cm)), ptr(prep(g_atmo)), ptr(prep(g_surf)), ptr(prep(g_w)),
                ptr(prep(g_alpha)), ptr(d_color), ptr(d_sigma), ptr(d_cs), ptr(d_z))
        call("anr_composite_bwd", *args, _lib.stream(dev))
        if d_z is not None:
            d_z = d_z.to(ctx.z_dtype)
        return d_z, d_color, d_sigma, d_cs, None, None


class _CompositeRef16Fn(torch.autograd.Function):
    """render_with_surface with the reference's f16 numerics (anr_composite_ref16_*)."""

    @staticmethod
    def forward(ctx, z, color, sigma, color_surf, z_scale: float, zero_rays, want16: bool):
        B, N, C = color.shape
        if sigma.shape[2] != 1:
            raise ANRError("reference-numerics composite: one density channel (B, N, 1)")
        dev = color.device
        color, sigma = color.contiguous(), sigma.contiguous()
        cs = color_surf.to(color.dtype).contiguous() if color_surf is not None else None
        zc = z.float().contiguous()
        f16 = torch.float16
        cm = torch.empty(B, C, device=dev, dtype=f16)
        atmo = torch.empty(B, C, device=dev, dtype=f16)
        surf = torch.empty(B, C, device=dev, dtype=f16) if cs is not None else None
        weights = torch.empty(B, N, 1, device=dev, dtype=f16)
        alpha = torch.empty(B, N, 1, device=dev, dtype=f16)
        c16 = torch.empty(B, N, C, device=dev, dtype=f16) if want16 else None
        s16 = torch.empty(B, N, 1, device=dev, dtype=f16) if want16 else None
        call("anr_composite_ref16_fwd", ptr(zc), float(z_scale), ptr(color), ptr(sigma), ptr(cs),
             dtype_code(color.dtype), B, N, C, ptr(cm), ptr(atmo), ptr(surf), ptr(weights),
             ptr(alpha), ptr(c16), ptr(s16), _lib.stream(dev), tag="composite_fwd")
        # the backward reads the inputs as f16 values either way: with the f16 copies at
        # hand it reads those (half the bytes of f32 inputs) and still returns gradients in
        # the inputs' dtype
        ctx.out_dtype = color.dtype
        if want16:
            ctx.save_for_backward(zc, c16, s16, cs)
        else:
            ctx.save_for_backward(zc, color, sigma, cs)
        ctx.set_materialize_grads(False)
        ctx.z_scale = float(z_scale)
        ctx.zero_rays = zero_rays
        outs = (cm, alpha, weights) if cs is None else (cm, alpha, weights, atmo, surf)
        if want16:
            ctx.mark_non_differentiable(c16, s16)
            outs = outs + (c16, s16)
        return outs

    @staticmethod
    def backward(ctx, g_cm, *unused):
        zc, color, sigma, cs = ctx.saved_tensors
        if any(g is not None for g in unused):
            raise ANRError("reference-numerics composite: gradients flow through color_map "
                           "only (as in the reference's loss)")
        B, N, C = color.shape
        dev = color.device
        if g_cm is None:
            g_cm = torch.zeros(B, C, device=dev, dtype=torch.float16)
        g_cm = g_cm.to(torch.float16).contiguous()
        od = ctx.out_dtype
        d_color = torch.empty(color.shape, device=dev, dtype=od)
        d_sigma = torch.empty(sigma.shape, device=dev, dtype=od)
        d_cs = (torch.empty(cs.shape, device=dev, dtype=od)
                if cs is not None and ctx.needs_input_grad[3] else None)
        if cs is not None and cs.dtype != color.dtype:
            cs = cs.to(color.dtype)
        call("anr_composite_ref16_bwd", ptr(zc), ctx.z_scale, ptr(color), ptr(sigma), ptr(cs),
             dtype_code(color.dtype), B, N, C, ptr(g_cm), ptr(d_color), ptr(d_sigma), ptr(d_cs),
             dtype_code(od), ptr(ctx.zero_rays), _lib.stream(dev), tag="composite_bwd")
        return None, d_color, d_sigma, d_cs, None, None, None


def render_with_surface_ref16(z_vals, color, sigma, color_surf, z_scale: float = 1.0,
                              zero_rays: torch.Tensor | None = None, inputs_f16: bool = False):
    """graphics_utils.py:52-77 with the reference's Instant-NGP numerics: z cast to f16
    (after the f32 ``z_vals * z_scale``), every op rounded to f16, torch's CUDA
    accumulation (f16 cumprod / cumsum, f32 sum / prod), and torch's f16 autograd as the
    backward (csrc/ref16.hip; restated in oracle/ref_f16.py). color / sigma / color_surf
    may be f32 (rounded to f16 on load, as a tcnn f16 output would be). Returns f16
    (color_map, alpha, weights, atmo, surf). ``zero_rays`` (int32 device tensor, optional)
    counts rays whose alpha rounded to exactly 1 in f16 (torch's zero-input backward
    branch, not reproduced: those rays get zero gradients). ``inputs_f16``: also return
    color and sigma rounded to f16 as the kernel reads them (tcnn's f16 outputs, which the
    reference's forward returns), written by the same kernel."""
    _check(z_vals, color, sigma)
    if zero_rays is None:
        zero_rays = torch.zeros(1, dtype=torch.int32, device=color.device)
    return _CompositeRef16Fn.apply(z_vals, color, sigma, color_surf, z_scale, zero_rays,
                                   bool(inputs_f16))


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
