"""Fused Instant-NGP radiance field: hash grid -> pos MLP -> dir encoding -> dir MLP.

One autograd node for the per-sample part of InstantNGPPipeline.forward
(src/atmonr/pipelines/instant_ngp.py:163-184):

    pos_enc = pos_encoder(pts)                          K3   (f16 table, f16 features)
    pos_out = pos_mlp(pos_enc)                          K6   (f16 MFMA, f32 out)
    dir_enc = dir_encoder(cat[dirs, pos_out[:, 1:]])    K5   (SH deg 2 | identity)
    color   = relu(dir_mlp(dir_enc))                    K6   (output ReLU in-kernel)
    sigma   = relu(pos_out[:, 0])

Inside the node the hash tables and MLP weights use the modules' compute dtype (f16 by
default, as tcnn) but every activation gradient crosses kernel boundaries in f32, so
none of the gradient chain underflows f16 (the reference's fp16-end-to-end autograd,
survey §0, loses small gradients; the f16 MLP backward here rescales per tile).
"""

from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call, dtype_code, ptr


class IngpFieldFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords, dirs, n_per_ray: int, p_hash, p_pos, p_dir, pipe):
        """coords (M,3) f32 in hash-grid space; dirs (B,3) f32, one per n_per_ray samples."""
        dev = coords.device
        s = _lib.stream(dev)
        M = coords.shape[0]
        enc_mod, pos_mod, dir_mod = pipe.pos_encoder, pipe.pos_mlp, pipe.dir_encoder
        dmlp = pipe.dir_mlp
        grid = enc_mod.hash_grids[0]
        cdt = pos_mod.dtype
        prec = _lib.F16 if cdt == torch.float16 else _lib.F32
        t_hash = p_hash.detach().to(enc_mod.dtype)
        w_pos = p_pos.detach().to(cdt)
        w_dir = p_dir.detach().to(cdt)

        enc = torch.empty(M, grid.n_out, device=dev, dtype=enc_mod.dtype)
        call("anr_hashgrid_fwd", ctypes.byref(grid.desc), ptr(coords), 3, M, ptr(t_hash),
             dtype_code(t_hash.dtype), ptr(enc), dtype_code(enc.dtype), enc.stride(0), s,
             tag="hash_fwd")
        pos_out = torch.empty(M, pos_mod.n_output_dims, device=dev, dtype=torch.float32)
        call("anr_mlp_fwd", ctypes.byref(pos_mod.desc), prec, ptr(w_pos), ptr(enc),
             dtype_code(enc.dtype), enc.stride(0), M, ptr(pos_out), _lib.F32,
             pos_out.stride(0), s, tag="pos_mlp_fwd")
        # dir encoding input: [SH(dir) | pos_out[:, 1:]]  (19 columns, tcnn pads to 32)
        n_sh = dir_mod.n_output_dims - (pos_mod.n_output_dims - 1)
        dir_in = torch.empty(M, dir_mod.n_output_dims, device=dev, dtype=cdt)
        dirs_rep = dirs.float().repeat_interleave(n_per_ray, dim=0)
        sh_leaf = dir_mod._leaves[0][1]
        call("anr_sh_fwd", sh_leaf.degree, ptr(dirs_rep), 3, M, ptr(dir_in), dtype_code(cdt),
             dir_in.stride(0), s)
        call("anr_identity", pos_out.data_ptr() + 4, _lib.F32, pos_out.stride(0), M,
             pos_mod.n_output_dims - 1, dir_in.data_ptr() + n_sh * dir_in.element_size(),
             dtype_code(cdt), dir_in.stride(0), s)
        color = torch.empty(M, dmlp.n_output_dims, device=dev, dtype=torch.float32)
        call("anr_mlp_fwd", ctypes.byref(pipe._dir_desc_relu), prec, ptr(w_dir), ptr(dir_in),
             dtype_code(cdt), dir_in.stride(0), M, ptr(color), _lib.F32, color.stride(0), s,
             tag="dir_mlp_fwd")
        sigma = torch.relu(pos_out[:, 0])
        ctx.save_for_backward(coords, enc, pos_out, dir_in, t_hash, w_pos, w_dir)
        ctx.pipe = pipe
        ctx.n_sh = n_sh
        return sigma, color

    @staticmethod
    def backward(ctx, d_sigma, d_color):
        coords, enc, pos_out, dir_in, t_hash, w_pos, w_dir = ctx.saved_tensors
        pipe = ctx.pipe
        dev = coords.device
        s = _lib.stream(dev)
        M = coords.shape[0]
        pos_mod, dmlp, enc_mod = pipe.pos_mlp, pipe.dir_mlp, pipe.pos_encoder
        grid = enc_mod.hash_grids[0]
        prec = _lib.F16 if pos_mod.dtype == torch.float16 else _lib.F32
        g_dir = torch.zeros(dmlp.params.shape, device=dev, dtype=torch.float32)
        g_pos = torch.zeros(pos_mod.params.shape, device=dev, dtype=torch.float32)
        g_hash = torch.zeros(enc_mod.params.shape, device=dev, dtype=torch.float32)
        if d_color is None:
            d_color = torch.zeros(M, dmlp.n_output_dims, device=dev)
        d_color = d_color.float().contiguous()
        d_dir_in = torch.empty(M, dir_in.shape[1], device=dev, dtype=torch.float32)
        call("anr_mlp_bwd", ctypes.byref(pipe._dir_desc_relu), prec, ptr(w_dir), ptr(dir_in),
             dtype_code(dir_in.dtype), dir_in.stride(0), M, ptr(d_color), _lib.F32,
             d_color.stride(0), ptr(d_dir_in), _lib.F32, d_dir_in.stride(0), ptr(g_dir), s,
             tag="dir_mlp_bwd")
        d_pos_out = torch.empty_like(pos_out)
        d_pos_out[:, 1:] = d_dir_in[:, ctx.n_sh:]
        if d_sigma is None:
            d_pos_out[:, 0] = 0
        else:
            d_pos_out[:, 0] = d_sigma.float() * (pos_out[:, 0] > 0)
        d_enc = torch.empty(M, enc.shape[1], device=dev, dtype=torch.float32)
        call("anr_mlp_bwd", ctypes.byref(pos_mod.desc), prec, ptr(w_pos), ptr(enc),
             dtype_code(enc.dtype), enc.stride(0), M, ptr(d_pos_out), _lib.F32,
             d_pos_out.stride(0), ptr(d_enc), _lib.F32, d_enc.stride(0), ptr(g_pos), s,
             tag="pos_mlp_bwd")
        call("anr_hashgrid_bwd", ctypes.byref(grid.desc), ptr(coords), 3, M, ptr(d_enc),
             _lib.F32, d_enc.stride(0), ptr(g_hash), s, tag="hash_bwd")
        return None, None, None, g_hash, g_pos, g_dir, None
