"""Fused Instant-NGP radiance field: hash grid -> pos MLP -> dir encoding -> dir MLP.

One autograd node for the per-sample part of InstantNGPPipeline.forward
(src/atmonr/pipelines/instant_ngp.py:163-184):

    pos_enc = pos_encoder(pts)                          K3   (f16 table, f16 features)
    pos_out = pos_mlp(pos_enc)                          K6   (f16 MFMA, f32 out)
    dir_enc = dir_encoder(cat[dirs, pos_out[:, 1:]])    \\
    color   = relu(dir_mlp(dir_enc))                    /  K6 with the dir encoding fused
    sigma   = relu(pos_out[:, 0])                          into its input loader

Inside the node the hash tables and MLP weights use the modules' compute dtype (f16 by
default, as tcnn) while every activation gradient crosses kernel boundaries in f32, so
the gradient chain does not underflow f16 (the reference's fp16 autograd does; survey
§0). The backward is three kernels: the dir-MLP backward writes dL/dpos_out directly
(density ReLU included), the pos-MLP backward writes dL/denc, the hash backward scatters
into the table gradient. When a parameter already has a float32 ``.grad`` (e.g. a
FlatGradBucket view), the kernels accumulate into it directly and the node returns no
gradient for that parameter — the same result as autograd's accumulation, one pass less.

With f16 networks of the shapes both reference configs use (pos 32->W->16, dir 19->W(x1|2)
->nb, W in {32, 64}) the two MLPs and the dir encoding run as ONE kernel each way
(anr_ingp_field_fwd/bwd): pos_out and dL/dpos_out stay in registers, the backward writes
only dL/denc. The weights are packed into MFMA fragment order once per forward. bf16
networks (BASELINE configs[4]: f16 hash features, bf16 MFMA MLP) run only this way.
The backward's workspace (per-wavefront f16 gradient maxima) is allocated here, through
torch's caching allocator, at anr_ingp_field_bwd_workspace_bytes.
"""

from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from ._lib import call, dtype_code, ptr


_grad_target = _lib.grad_target


def _done(*pairs) -> None:
    """_lib.grad_done for each (direct, param) pair whose gradient was written directly."""
    for direct, p in zip(pairs[::2], pairs[1::2]):
        if direct:
            _lib.grad_done(p)


class IngpFieldFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords, dirs, n_per_ray: int, p_hash, p_pos, p_dir, pipe, rows=None,
                m_dense: int = 0):
        """coords (M,3) f32 in hash-grid space; dirs (B,3) f32, one per n_per_ray samples.
        With ``rows`` (occupancy culling, atmonr_amd.occupancy): coords are the kept
        samples, rows (M,) int32 their indices among the m_dense ray-major samples; sigma
        and color come back dense (m_dense rows), zero at the culled samples."""
        dev = coords.device
        s = _lib.stream(dev)
        M = coords.shape[0]
        enc_mod, pos_mod = pipe.pos_encoder, pipe.pos_mlp
        grid = enc_mod.hash_grids[0]
        cdt = pos_mod.dtype
        prec = _lib.F16 if cdt == torch.float16 else _lib.F32
        t_hash = _lib.compute_copy(p_hash, enc_mod.dtype)
        dirs = dirs.float().contiguous()

        fused = field_fused(pipe) and enc_mod.dtype == torch.float16
        if rows is not None and not fused:
            raise _lib.ANRError("occupancy culling needs the fused f16 field")
        if cdt == torch.bfloat16 and not fused:
            raise _lib.ANRError("bf16 networks run only in the fused field (f16 hash features)")
        ctx.pipe = pipe
        ctx.n_per_ray = n_per_ray
        ctx.params = (p_hash, p_pos, p_dir)
        ctx.rows = rows
        planes = fused and _enc_planes(grid, M)
        if fused:
            mma = _mma_code(pipe)
            pdesc, ddesc = ctypes.byref(pos_mod.desc), ctypes.byref(pipe.dir_mlp.desc)
            packed = torch.empty(_lib.load().anr_ingp_field_packed_size(pdesc, ddesc),
                                 device=dev, dtype=torch.float16)  # 16-bit carrier
            m_pos, m_dir = _lib.pack_source(p_pos, mma), _lib.pack_source(p_dir, mma)
            call("anr_ingp_field_pack", pdesc, ddesc, mma, ptr(m_pos), ptr(m_dir), ptr(packed),
                 s, tag="field_pack")
            nb = pipe.dir_mlp.n_output_dims
        if planes and rows is None and _hash_field_ok(grid, nb, n_per_ray):
            # hash grid + field forward in one kernel (anr_ingp_hash_field_fwd): the level-
            # quad planes are written for the backward and never re-read by the forward
            nq = (grid.desc.n_levels + 3) // 4
            enc = torch.empty(nq, M, 8, device=dev, dtype=torch.float16)
            ctx.enc_ld = -8 * M
            sigma = torch.empty(M, device=dev, dtype=torch.float32)
            color = torch.empty(M, nb, device=dev, dtype=torch.float32)
            call("anr_ingp_hash_field_fwd", ctypes.byref(grid.desc), ptr(coords), M,
                 ptr(t_hash), dtype_code(t_hash.dtype), ptr(enc), 8 * M, pdesc, ddesc, mma,
                 ptr(packed), ptr(dirs), n_per_ray, ptr(sigma), ptr(color), color.stride(0), s,
                 tag="hash_field_fwd")
            ctx.fused_field = True
            ctx.save_for_backward(coords, dirs, enc, packed)
            return sigma, color
        if planes:
            # level-quad planes (anr_hashgrid_fwd_planes: one lane per sample, coalesced;
            # 0.47-0.50 ms vs the row-layout walker's 0.63 at the bench shape), handed to the
            # field kernels as enc_stride = -plane
            nq = (grid.desc.n_levels + 3) // 4
            enc = torch.empty(nq, M, 8, device=dev, dtype=torch.float16)
            enc_ld = -8 * M
            call("anr_hashgrid_fwd_planes", ctypes.byref(grid.desc), ptr(coords), 3, M,
                 ptr(t_hash), dtype_code(t_hash.dtype), ptr(enc), 8 * M, s, tag="hash_fwd")
        else:
            enc = torch.empty(M, grid.n_out, device=dev, dtype=enc_mod.dtype)
            enc_ld = enc.stride(0)
            call("anr_hashgrid_fwd", ctypes.byref(grid.desc), ptr(coords), 3, M, ptr(t_hash),
                 dtype_code(t_hash.dtype), ptr(enc), dtype_code(enc.dtype), enc_ld, s,
                 tag="hash_fwd")
        ctx.enc_ld = enc_ld
        if fused:
            if rows is None:
                sigma = torch.empty(M, device=dev, dtype=torch.float32)
                color = torch.empty(M, nb, device=dev, dtype=torch.float32)
                call("anr_ingp_field_fwd", pdesc, ddesc, mma, ptr(packed), ptr(enc), enc_ld,
                     ptr(dirs), n_per_ray, M, ptr(sigma), ptr(color), color.stride(0), s,
                     tag="field_fwd")
            else:
                sigma = torch.zeros(m_dense, device=dev, dtype=torch.float32)
                color = torch.zeros(m_dense, nb, device=dev, dtype=torch.float32)
                call("anr_ingp_field_fwd_rows", pdesc, ddesc, mma, ptr(packed), ptr(enc),
                     enc_ld, ptr(dirs), n_per_ray, M, ptr(rows), ptr(sigma), ptr(color),
                     color.stride(0), s, tag="field_fwd")
            ctx.fused_field = True
            ctx.save_for_backward(coords, dirs, enc, packed)
            return sigma, color
        ctx.fused_field = False
        w_pos = _lib.compute_copy(p_pos, cdt)
        w_dir = _lib.compute_copy(p_dir, cdt)
        pos_out = torch.empty(M, pos_mod.n_output_dims, device=dev, dtype=torch.float32)
        call("anr_mlp_fwd", ctypes.byref(pos_mod.desc), prec, ptr(w_pos), ptr(enc),
             dtype_code(enc.dtype), enc.stride(0), M, ptr(pos_out), _lib.F32,
             pos_out.stride(0), s, tag="pos_mlp_fwd")
        color = torch.empty(M, pipe.dir_mlp.n_output_dims, device=dev, dtype=torch.float32)
        call("anr_ingp_dir_mlp_fwd", ctypes.byref(pipe._dir_desc_relu), prec, ptr(w_dir),
             ptr(pos_out), pos_out.stride(0), ptr(dirs), n_per_ray, M, ptr(color), _lib.F32,
             color.stride(0), s, tag="dir_mlp_fwd")
        sigma = torch.relu(pos_out[:, 0])
        ctx.save_for_backward(coords, dirs, enc, pos_out, w_pos, w_dir)
        return sigma, color

    @staticmethod
    def backward(ctx, d_sigma, d_color):
        if ctx.fused_field:
            return IngpFieldFn._backward_fused(ctx, d_sigma, d_color)
        coords, dirs, enc, pos_out, w_pos, w_dir = ctx.saved_tensors
        pipe = ctx.pipe
        dev = coords.device
        s = _lib.stream(dev)
        M = coords.shape[0]
        pos_mod, enc_mod = pipe.pos_mlp, pipe.pos_encoder
        grid = enc_mod.hash_grids[0]
        prec = _lib.F16 if pos_mod.dtype == torch.float16 else _lib.F32
        p_hash, p_pos, p_dir = ctx.params
        g_hash, direct_h = _grad_target(p_hash, dev)
        g_pos, direct_p = _grad_target(p_pos, dev)
        g_dir, direct_d = _grad_target(p_dir, dev)
        if d_color is None:
            d_color = torch.zeros(M, pipe.dir_mlp.n_output_dims, device=dev)
        d_color = d_color.float().contiguous()
        d_sigma = d_sigma.float().contiguous() if d_sigma is not None else None
        d_pos_out = torch.empty_like(pos_out)
        call("anr_ingp_dir_mlp_bwd", ctypes.byref(pipe._dir_desc_relu), prec, ptr(w_dir),
             ptr(pos_out), pos_out.stride(0), ptr(dirs), ctx.n_per_ray, M, ptr(d_color),
             d_color.stride(0), ptr(d_sigma), ptr(d_pos_out), d_pos_out.stride(0), ptr(g_dir),
             s, tag="dir_mlp_bwd")
        d_enc = torch.empty(M, pipe.pos_encoder.hash_grids[0].n_out, device=dev, dtype=torch.float32)
        call("anr_mlp_bwd", ctypes.byref(pos_mod.desc), prec, ptr(w_pos), ptr(enc),
             dtype_code(enc.dtype), enc.stride(0), M, ptr(d_pos_out), _lib.F32,
             d_pos_out.stride(0), ptr(d_enc), _lib.F32, d_enc.stride(0), ptr(g_pos), s,
             tag="pos_mlp_bwd")
        call("anr_hashgrid_bwd", ctypes.byref(grid.desc), ptr(coords), 3, M, ptr(d_enc),
             _lib.F32, d_enc.stride(0), ptr(g_hash), s, tag="hash_bwd")
        _done(direct_d, p_dir, direct_p, p_pos, direct_h, p_hash)
        return (None, None, None, None if direct_h else g_hash, None if direct_p else g_pos,
                None if direct_d else g_dir, None, None, None)

    @staticmethod
    def _backward_fused(ctx, d_sigma, d_color):
        coords, dirs, enc, packed = ctx.saved_tensors
        pipe = ctx.pipe
        dev = coords.device
        s = _lib.stream(dev)
        M = coords.shape[0]
        grid = pipe.pos_encoder.hash_grids[0]
        p_hash, p_pos, p_dir = ctx.params
        g_hash, direct_h = _grad_target(p_hash, dev)
        g_pos, direct_p = _grad_target(p_pos, dev)
        g_dir, direct_d = _grad_target(p_dir, dev)
        if d_color is None:
            d_color = torch.zeros(M, pipe.dir_mlp.n_output_dims, device=dev)
        d_color = d_color.float().contiguous()
        d_sigma = d_sigma.float().contiguous() if d_sigma is not None else None
        n_enc = pipe.pos_encoder.hash_grids[0].n_out
        pdesc, ddesc = ctypes.byref(pipe.pos_mlp.desc), ctypes.byref(pipe.dir_mlp.desc)
        mma = _mma_code(pipe)
        ls = getattr(pipe, "loss_scale", None)
        tiles = row_nz = None
        if ls and _ROW_BITS and not _TILE_SKIP and n_enc == 32 and ctx.rows is None:
            # reference numerics (default since r06): dL/denc as f16 rows, the values
            # tinycudann hands the hash grid (exactly f16 numbers), plus one bit per row with
            # a nonzero value; the hash-grid backward loads and walks only those rows
            # (~27 % of them once training settles). ANR_ROW_BITS=0: f32 rows, every row
            # loaded, the per-sample zero test (the r05 form, A/B)
            d_enc = torch.empty(M, n_enc, device=dev, dtype=torch.float16)
            row_nz = torch.empty((M + 31) // 32, device=dev, dtype=torch.int32)
            # with a workspace: a pos pass over the tiles whose dL/dcolor is zero (every tile
            # once training settles: the dir network adds exactly 0 there) at two waves per
            # SIMD, and a full pass over the tiles it lists. ANR_POS_PASS=0: one kernel
            ws_bytes = _lib.load().anr_ingp_field_bwd_ref16_rows_workspace_bytes(M) if _POS_PASS else 0
            ws = torch.empty(max(1, ws_bytes), device=dev, dtype=torch.uint8) if ws_bytes else None
            call("anr_ingp_field_bwd_ref16_rows", pdesc, ddesc, ptr(packed), ptr(enc),
                 ctx.enc_ld, ptr(dirs), ctx.n_per_ray, M, ptr(d_sigma), ptr(d_color),
                 d_color.stride(0), ptr(d_enc), d_enc.stride(0), ptr(g_pos), ptr(g_dir),
                 float(ls), ptr(row_nz), None if ws is None else ptr(ws), ws_bytes, s,
                 tag="field_bwd")
        elif ls:
            d_enc = torch.empty(M, n_enc, device=dev, dtype=torch.float32)
            # reference numerics: tcnn's loss-scaled f16 backward. ANR_TILE_SKIP=1: it also
            # marks the 32-row tiles whose incoming gradients are all zero and the hash-grid
            # backward skips them without loading. Off by default: measured no faster than
            # the per-sample skip alone (2.782 vs 2.769 ms/step, profiles/r05_tile_skip_ab.log)
            if ctx.rows is not None:
                raise _lib.ANRError("reference numerics: no occupancy culling")
            if _TILE_SKIP:
                tiles = torch.empty((M + 31) // 32, device=dev, dtype=torch.uint8)
                call("anr_ingp_field_bwd_ref16_tiles", pdesc, ddesc, ptr(packed), ptr(enc),
                     ctx.enc_ld, ptr(dirs), ctx.n_per_ray, M, ptr(d_sigma), ptr(d_color),
                     d_color.stride(0), ptr(d_enc), d_enc.stride(0), ptr(g_pos), ptr(g_dir),
                     float(ls), ptr(tiles), s, tag="field_bwd")
            else:
                call("anr_ingp_field_bwd_ref16", pdesc, ddesc, ptr(packed), ptr(enc),
                     ctx.enc_ld, ptr(dirs), ctx.n_per_ray, M, ptr(d_sigma), ptr(d_color),
                     d_color.stride(0), ptr(d_enc), d_enc.stride(0), ptr(g_pos), ptr(g_dir),
                     float(ls), s, tag="field_bwd")
        else:
            d_enc = torch.empty(M, n_enc, device=dev, dtype=torch.float32)
            ws_bytes = _lib.load().anr_ingp_field_bwd_workspace_bytes(pdesc, ddesc, mma, M)
            ws = torch.empty(max(1, -(-ws_bytes // 4)), device=dev, dtype=torch.float32)
            if ctx.rows is None:
                call("anr_ingp_field_bwd", pdesc, ddesc, mma, ptr(packed), ptr(enc),
                     ctx.enc_ld, ptr(dirs), ctx.n_per_ray, M, ptr(d_sigma), ptr(d_color),
                     d_color.stride(0), ptr(d_enc), d_enc.stride(0), ptr(g_pos), ptr(g_dir),
                     ptr(ws), ws_bytes, s, tag="field_bwd")
            else:  # dL/d(sigma, color) are dense; read at the kept samples' rows
                call("anr_ingp_field_bwd_rows", pdesc, ddesc, mma, ptr(packed), ptr(enc),
                     ctx.enc_ld, ptr(dirs), ctx.n_per_ray, M, ptr(ctx.rows), ptr(d_sigma),
                     ptr(d_color), d_color.stride(0), ptr(d_enc), d_enc.stride(0), ptr(g_pos),
                     ptr(g_dir), ptr(ws), ws_bytes, s, tag="field_bwd")
        _done(direct_p, p_pos, direct_d, p_dir)  # MLP grads final: their all-reduce may start
        if getattr(pipe, "_keep_d_enc", False):
            # diagnostics (tools/ref16_field_diag.py) and bench.py's request count of this
            # hash-grid backward (anr_hashgrid_bwd_count_requests on the same inputs)
            pipe._last_d_enc = d_enc
            pipe._last_hash_bwd = (coords, d_enc, g_hash)
            pipe._last_field_grads = (d_sigma, d_color)
        if row_nz is not None:
            call("anr_hashgrid_bwd_rows", ctypes.byref(grid.desc), ptr(coords), 3, M,
                 ptr(d_enc), _lib.F16, d_enc.stride(0), ptr(g_hash), ptr(row_nz), s,
                 tag="hash_bwd")
        elif tiles is not None:
            call("anr_hashgrid_bwd_tiles", ctypes.byref(grid.desc), ptr(coords), 3, M,
                 ptr(d_enc), _lib.F32, d_enc.stride(0), ptr(g_hash), ptr(tiles), s,
                 tag="hash_bwd")
        else:
            call("anr_hashgrid_bwd", ctypes.byref(grid.desc), ptr(coords), 3, M, ptr(d_enc),
                 _lib.F32, d_enc.stride(0), ptr(g_hash), s, tag="hash_bwd")
        _done(direct_h, p_hash)
        return (None, None, None, None if direct_h else g_hash, None if direct_p else g_pos,
                None if direct_d else g_dir, None, None, None)


def _mma_code(pipe) -> int:
    return _lib.BF16 if pipe.pos_mlp.dtype == torch.bfloat16 else _lib.F16


def _enc_planes(grid, M: int) -> bool:
    """The fused field reads the hash features as level-quad planes (default) or, with
    ANR_ENC_PLANES=0 (A/B), in the row layout of the walker forward. The planes kernel
    addresses its output with 32-bit byte offsets (16 B per sample and quad): above ~33 M
    samples at 16 levels the row layout (whose walker falls back to 64-bit indexing) runs."""
    d = grid.desc
    nq = (d.n_levels + 3) // 4
    return (_ENC_PLANES and d.n_features == 2 and d.n_levels <= 16 and d.n_dims == 3
            and 16 * nq * (M + 256) < 2 ** 31)


def _hash_field_ok(grid, n_out: int, n_per_ray: int) -> bool:
    """anr_ingp_hash_field_fwd's shapes: 16 levels x 2 features (3-D), 4 colour outputs,
    samples per ray a multiple of 64. ANR_HASH_FIELD=0 keeps the two-kernel forward (A/B)."""
    d = grid.desc
    return (_HASH_FIELD and d.n_levels == 16 and d.n_features == 2 and d.n_dims == 3
            and n_out == 4 and n_per_ray % 64 == 0)


_ENC_PLANES = os.environ.get("ANR_ENC_PLANES", "1") != "0"
_HASH_FIELD = os.environ.get("ANR_HASH_FIELD", "0") != "0"
_TILE_SKIP = os.environ.get("ANR_TILE_SKIP", "0") != "0"
_ROW_BITS = os.environ.get("ANR_ROW_BITS", "1") != "0"
_POS_PASS = os.environ.get("ANR_POS_PASS", "1") != "0"


def field_fused(pipe) -> bool:
    """True when the pipeline's networks run through anr_ingp_field_{fwd,bwd}."""
    flag = getattr(pipe, "_field_fused", None)
    if flag is None:
        ok = (pipe.pos_mlp.dtype in (torch.float16, torch.bfloat16)
              and pipe.dir_mlp.dtype == pipe.pos_mlp.dtype
              and (pipe.pos_mlp.dtype == torch.float16
                   or pipe.pos_encoder.dtype == torch.float16)
              and getattr(pipe, "allow_field_fusion", True)
              and getattr(pipe, "fused", True))  # fused=False: the unfused parity path
        if ok:
            ok = bool(_lib.load().anr_ingp_field_supported(ctypes.byref(pipe.pos_mlp.desc),
                                                           ctypes.byref(pipe.dir_mlp.desc)))
        pipe._field_fused = flag = ok
    return flag


@torch.no_grad()
def field_density(pipe, pts: torch.Tensor, run_length: int = 0) -> torch.Tensor:
    """sigma = relu(pos_mlp(pos_encoder(pts))[:, 0]) at hash-grid points (P, 3) through the
    fused kernels (hash forward, then anr_ingp_field_density: the pos MLP of
    anr_ingp_field_fwd without the dir MLP, bit-identical sigma). The extract path of
    instant_ngp.py:208-247 and the occupancy grid's density function, for pipelines whose
    field is fused (the only path for bf16 networks). ``run_length``: the points come in
    runs of that many spatial neighbours (an extract column's altitudes), which the
    hash-grid walker's chunks then follow (anr_hashgrid_fwd_runs; same values)."""
    dev = pts.device
    s = _lib.stream(dev)
    P = pts.shape[0]
    sigma = torch.empty(P, device=dev, dtype=torch.float32)
    if P == 0:
        return sigma
    enc_mod, pos_mod = pipe.pos_encoder, pipe.pos_mlp
    grid = enc_mod.hash_grids[0]
    pts = pts.float().contiguous()
    t_hash = _lib.compute_copy(enc_mod.params, enc_mod.dtype)
    enc = torch.empty(P, grid.n_out, device=dev, dtype=torch.float16)
    call("anr_hashgrid_fwd_runs", ctypes.byref(grid.desc), ptr(pts), 3, P, int(run_length),
         ptr(t_hash), dtype_code(t_hash.dtype), ptr(enc), _lib.F16, enc.stride(0), s,
         tag="hash_fwd")
    mma = _mma_code(pipe)
    pdesc, ddesc = ctypes.byref(pos_mod.desc), ctypes.byref(pipe.dir_mlp.desc)
    packed = torch.empty(_lib.load().anr_ingp_field_packed_size(pdesc, ddesc), device=dev,
                         dtype=torch.float16)
    call("anr_ingp_field_pack", pdesc, ddesc, mma, ptr(_lib.pack_source(pos_mod.params, mma)),
         ptr(_lib.pack_source(pipe.dir_mlp.params, mma)), ptr(packed), s, tag="field_pack")
    # the pos MLP only (anr_ingp_field_density): sigma bit-identical to the full field's
    call("anr_ingp_field_density", pdesc, ddesc, mma, ptr(packed), ptr(enc), enc.stride(0), P,
         ptr(sigma), s, tag="field_density")
    return sigma
