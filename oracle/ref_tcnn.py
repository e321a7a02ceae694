"""ORACLE (test infrastructure only): tiny-cuda-nn module semantics restated on CPU.

The reference calls tinycudann (unpinned, installed from git HEAD per README.md:19-22,
not vendored) at src/atmonr/pipelines/instant_ngp.py:60-85 (construction) and
:163-174, :236-237 (calls). tcnn is absent here, so these functions restate its
published algorithm:

* GridEncoding (HashGrid), tcnn include/tiny-cuda-nn/encodings/grid.h: level scale
  2^(l log2 s) * base - 1, resolution ceil(scale)+1, fma(scale, x, 0.5) positions,
  dense strided index while the stride fits the level's table, else the XOR prime hash
  (1, 2654435761, 805459861), modulo the level size; per-level sizes
  min(next_multiple(res^D, 8), 2^log2T). Linear interpolation.
* SphericalHarmonics: input remapped 2x-1, degree d -> d^2 standard real SH terms.
* Composite / Identity; encodings padded with 1.0 to the network width.
* FullyFusedMLP: bias-free, ReLU hidden, output padded to 16 and sliced.

Parity of these pieces against real tcnn is UNPINNED (no tcnn outputs exist offline);
they are pinned by the known-answer tests in tests/test_oracle_tcnn.py.
"""

from __future__ import annotations

import math

import numpy as np
import torch

PRIMES = np.array([1, 2654435761, 805459861], dtype=np.uint32)


def grid_levels(n_dims, n_levels, base_resolution, per_level_scale, log2_hashmap_size):
    """Per-level (offset, size, resolution, scale) exactly as tcnn's GridEncoding."""
    log2_pls = np.float32(math.log2(np.float32(per_level_scale)))
    offsets, sizes, res, scales = [], [], [], []
    off = 0
    for lvl in range(n_levels):
        s = np.float32(np.float32(2.0) ** (np.float32(lvl) * log2_pls)) * np.float32(
            base_resolution
        ) - np.float32(1.0)
        s = np.float32(s)
        r = int(math.ceil(float(s))) + 1
        n = r**n_dims
        n = (n + 7) // 8 * 8
        n = min(n, 1 << log2_hashmap_size)
        offsets.append(off)
        sizes.append(n)
        res.append(r)
        scales.append(s)
        off += n
    return np.array(offsets), np.array(sizes), np.array(res), np.array(scales, np.float32), off


def grid_index(cells: np.ndarray, T: int, res: int) -> np.ndarray:
    """cells: (M, D) uint32 -> (M,) uint32 table index within the level."""
    D = cells.shape[1]
    stride = 1
    index = np.zeros(cells.shape[0], dtype=np.uint32)
    d = 0
    while d < D and stride <= T:
        index = index + cells[:, d] * np.uint32(stride)
        stride *= res
        d += 1
    if T < stride:
        index = np.zeros(cells.shape[0], dtype=np.uint32)
        for d in range(D):
            index ^= cells[:, d] * PRIMES[d]
    return index % np.uint32(T)


def _positions(x: np.ndarray, scale: np.float32):
    p = (np.float64(scale) * x.astype(np.float64) + 0.5).astype(np.float32)
    cell_f = np.floor(p)
    w = (p - cell_f).astype(np.float64)
    cells = cell_f.astype(np.int64).astype(np.uint32)
    return cells, w


def hashgrid_corners(x, cfg, level):
    """Per-sample corner indices (M, 2^D) and weights (M, 2^D) for one level."""
    offsets, sizes, res, scales, _ = grid_levels(*cfg)
    cells, w = _positions(x, scales[level])
    D = x.shape[1]
    idx = np.zeros((x.shape[0], 1 << D), dtype=np.int64)
    wt = np.ones((x.shape[0], 1 << D), dtype=np.float64)
    for c in range(1 << D):
        gc = cells.copy()
        for d in range(D):
            if (c >> d) & 1:
                gc[:, d] = gc[:, d] + np.uint32(1)
                wt[:, c] *= w[:, d]
            else:
                wt[:, c] *= 1.0 - w[:, d]
        idx[:, c] = offsets[level] + grid_index(gc, int(sizes[level]), int(res[level])).astype(
            np.int64
        )
    return idx, wt


def hashgrid_fwd(x: np.ndarray, table: np.ndarray, cfg, n_features: int = 2) -> np.ndarray:
    """x (M, D) in [0,1]; table (n_entries*F,) -> (M, L*F) float64."""
    n_levels = cfg[1]
    tab = table.astype(np.float64).reshape(-1, n_features)
    out = np.zeros((x.shape[0], n_levels * n_features))
    for lvl in range(n_levels):
        idx, wt = hashgrid_corners(x, cfg, lvl)
        out[:, lvl * n_features:(lvl + 1) * n_features] = np.einsum("mc,mcf->mf", wt, tab[idx])
    return out


def hashgrid_bwd(x: np.ndarray, dout: np.ndarray, cfg, n_entries: int, n_features: int = 2):
    n_levels = cfg[1]
    grad = np.zeros((n_entries, n_features))
    for lvl in range(n_levels):
        idx, wt = hashgrid_corners(x, cfg, lvl)
        g = dout[:, lvl * n_features:(lvl + 1) * n_features].astype(np.float64)
        contrib = wt[:, :, None] * g[:, None, :]
        np.add.at(grad, idx.reshape(-1), contrib.reshape(-1, n_features))
    return grad.reshape(-1)


def sh(x: np.ndarray, degree: int) -> np.ndarray:
    """tcnn SphericalHarmonics on x in [0,1]^3 (remapped to 2x-1)."""
    x = x.astype(np.float64) * 2.0 - 1.0
    X, Y, Z = x[:, 0], x[:, 1], x[:, 2]
    terms = [np.full_like(X, 0.28209479177387814)]
    if degree > 1:
        terms += [-0.48860251190291987 * Y, 0.48860251190291987 * Z, -0.48860251190291987 * X]
    if degree > 2:
        terms += [
            1.0925484305920792 * X * Y,
            -1.0925484305920792 * Y * Z,
            0.94617469575755997 * Z * Z - 0.31539156525251999,
            -1.0925484305920792 * X * Z,
            0.54627421529603959 * X * X - 0.54627421529603959 * Y * Y,
        ]
    if degree > 3:
        terms += [
            0.59004358992664352 * Y * (-3.0 * X * X + Y * Y),
            2.8906114426405538 * X * Y * Z,
            0.45704579946446572 * Y * (1.0 - 5.0 * Z * Z),
            0.3731763325901154 * Z * (5.0 * Z * Z - 3.0),
            0.45704579946446572 * X * (1.0 - 5.0 * Z * Z),
            1.4453057213202769 * Z * (X * X - Y * Y),
            0.59004358992664352 * X * (-X * X + 3.0 * Y * Y),
        ]
    return np.stack(terms, axis=1)


def mlp_layer_shapes(n_in, n_out, width, n_hidden):
    nip = (n_in + 15) // 16 * 16
    nop = (n_out + 15) // 16 * 16
    shapes = [(width, nip)] + [(width, width)] * (n_hidden - 1) + [(nop, width)]
    return shapes, nip, nop


class _RoundValue(torch.autograd.Function):
    """x -> float64(dtype(x)) forward; the gradient passes through UNCHANGED. (A plain
    ``t.half().double()`` is not that: autograd casts the incoming gradient back through
    f16, quantising small unscaled gradients -- the r02 oracle's f16 "exact" gradients
    were rounded that way.)"""

    @staticmethod
    def forward(ctx, x, dtype):
        return x.to(dtype).double()

    @staticmethod
    def backward(ctx, g):
        return g, None


class ReluRound(torch.autograd.Function):
    """relu(x) rounded to ``dtype`` (a hidden activation of an f16 / bf16 MLP tile). The
    backward masks with the ROUNDED output, as tcnn's ReLU backward tests the stored f16
    activation > 0 (so a pre-activation below the f16 subnormal range passes no
    gradient); ``round_grad`` also rounds the gradient to ``dtype`` (tcnn's f16 gradient
    tiles, reference semantics), else it passes in full precision."""

    @staticmethod
    def forward(ctx, x, dtype, round_grad):
        y = torch.relu(x).to(dtype).to(x.dtype)
        ctx.save_for_backward(y)
        ctx.dtype, ctx.round_grad = dtype, round_grad
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        g = torch.where(y > 0, g, torch.zeros_like(g))
        if ctx.round_grad:
            g = g.to(ctx.dtype).to(y.dtype)
        return g, None, None


def relu_rounder(half, round_grad: bool = False):
    """Hidden-layer ReLU + rounding of an MLP tile: identity rounding for half=False."""
    if not half:
        return torch.relu
    dt = torch.bfloat16 if half == "bf16" else torch.float16
    return lambda t: ReluRound.apply(t, dt, round_grad)


def rounder(half):
    """float64 -> the kernel's 16-bit operand type -> float64 on the VALUES (identity for
    half=False); gradients flow through in full precision."""
    if half == "bf16":
        return lambda t: _RoundValue.apply(t, torch.bfloat16)
    if half:
        return lambda t: _RoundValue.apply(t, torch.float16)
    return lambda t: t


def mlp_fwd(x: torch.Tensor, params: torch.Tensor, n_in, n_out, width, n_hidden,
            output_relu=False, half=False) -> torch.Tensor:
    """tcnn FullyFusedMLP in float64 (autograd-capable). half=True rounds the inputs,
    weights and every hidden activation to float16 like the f16 kernel does; half="bf16"
    rounds them to bfloat16 instead (the build's bf16 MFMA field, BASELINE configs[4],
    which has no tcnn counterpart)."""
    shapes, nip, nop = mlp_layer_shapes(n_in, n_out, width, n_hidden)
    rnd = rounder(half)
    h = torch.ones(x.shape[0], nip, dtype=torch.float64)
    h = torch.cat([rnd(x.double()), h[:, n_in:]], dim=1)
    off = 0
    act = relu_rounder(half)
    for k, (o, i) in enumerate(shapes):
        W = rnd(params[off:off + o * i].double()).view(o, i)
        off += o * i
        h = h @ W.t()
        if k < len(shapes) - 1:
            h = act(h)  # relu, rounded; backward masks on the rounded activation
        elif output_relu:
            h = torch.relu(h)
    return h[:, :n_out]
