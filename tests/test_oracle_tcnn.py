"""Known-answer tests pinning the tiny-cuda-nn restatement (oracle/ref_tcnn.py).

tcnn is not in /root/reference and cannot be installed offline, so these tests encode
its published semantics by hand: table sizes, dense vs hashed indexing, trilinear
weights, SH values, MLP padding. CPU only."""

import numpy as np
import torch

from oracle import ref_tcnn

CFG_POS21 = (3, 16, 16, 1.3819, 21)
CFG_POS19 = (3, 16, 16, 1.3819, 19)
CFG_SURF = (2, 16, 16, 1.3819, 19)


def test_table_sizes_match_survey():
    # 42,283,392 (T=2^21), 12,196,240 (T=2^19), 5,522,000 (2-D T=2^19)
    for cfg, n in [(CFG_POS21, 42_283_392), (CFG_POS19, 12_196_240), (CFG_SURF, 5_522_000)]:
        *_, entries = ref_tcnn.grid_levels(*cfg)
        assert entries * 2 == n


def test_resolutions():
    _, _, res, _, _ = ref_tcnn.grid_levels(*CFG_POS21)
    assert res.tolist() == [16, 23, 31, 43, 59, 81, 112, 154, 213, 295, 407, 562, 776, 1073,
                            1482, 2048]


def test_dense_and_hashed_index_by_hand():
    # dense level: index = x + y*res + z*res^2
    cells = np.array([[3, 4, 5], [15, 0, 1]], dtype=np.uint32)
    idx = ref_tcnn.grid_index(cells, T=4096, res=16)
    assert idx.tolist() == [3 + 4 * 16 + 5 * 256, 15 + 0 + 256]
    # hashed level: (x*1 ^ y*2654435761 ^ z*805459861) mod T, uint32 wrap-around
    T = 1 << 19
    x, y, z = 1000, 777, 12
    h = (x ^ ((y * 2654435761) & 0xFFFFFFFF) ^ ((z * 805459861) & 0xFFFFFFFF)) % T
    idx = ref_tcnn.grid_index(np.array([[x, y, z]], dtype=np.uint32), T=T, res=2048)
    assert idx.tolist() == [h]


def test_trilinear_single_point():
    cfg = (3, 1, 16, 1.3819, 19)  # one level: res 16, scale 15
    x = np.array([[0.1, 0.5, 0.9]], dtype=np.float32)
    idx, wt = ref_tcnn.hashgrid_corners(x, cfg, 0)
    # fma(scale, x, 0.5) rounds once to f32 (z: 15*0.9f + 0.5 = 13.9999996 -> 14.0f)
    p = (15.0 * x[0].astype(np.float64) + 0.5).astype(np.float32).astype(np.float64)
    c = np.floor(p)
    f = p - c
    assert c.tolist() == [2.0, 8.0, 14.0]
    assert np.isclose(wt.sum(), 1.0)
    # corner 0 = (c0, c1, c2) with weight prod(1 - f); corner 7 = (c+1) with prod(f)
    assert idx[0, 0] == int(c[0] + c[1] * 16 + c[2] * 256)
    assert np.isclose(wt[0, 0], np.prod(1 - f))
    assert np.isclose(wt[0, 7], np.prod(f))
    # features: table value = entry index -> interpolated value = sum(w * idx)
    table = np.repeat(np.arange(16**3, dtype=np.float32), 2)
    out = ref_tcnn.hashgrid_fwd(x, table, cfg)
    assert np.isclose(out[0, 0], (wt * idx).sum())


def test_hashgrid_bwd_is_adjoint_of_fwd():
    rng = np.random.default_rng(0)
    cfg = (3, 6, 4, 1.6, 10)
    *_, entries = ref_tcnn.grid_levels(*cfg)
    x = rng.random((300, 3), dtype=np.float32)
    table = rng.standard_normal(entries * 2)
    g = rng.standard_normal((300, 12))
    lhs = (ref_tcnn.hashgrid_fwd(x, table, cfg) * g).sum()
    rhs = (table * ref_tcnn.hashgrid_bwd(x, g, cfg, entries)).sum()
    assert np.isclose(lhs, rhs, rtol=1e-10)


def test_sh_degree2_known_values():
    # +z direction (x in [0,1] coords -> (0.5, 0.5, 1.0)): [Y00, -c*y, c*z, -c*x] = [.2821, 0, .4886, 0]
    out = ref_tcnn.sh(np.array([[0.5, 0.5, 1.0]]), 2)
    assert np.allclose(out, [[0.28209479177387814, 0.0, 0.48860251190291987, 0.0]])
    # degree 4 on a unit vector: sum of squares of all terms = 4 / (4*pi) * ... (Unsold)
    v = np.array([[0.3, -0.5, 0.8]])
    v = v / np.linalg.norm(v)
    out = ref_tcnn.sh((v + 1) / 2, 4)
    assert np.isclose((out**2).sum(), 16 / (4 * np.pi))


def test_mlp_padding_is_ones_and_output_sliced():
    n_in, n_out, width = 19, 4, 32
    shapes, nip, nop = ref_tcnn.mlp_layer_shapes(n_in, n_out, width, 2)
    assert (nip, nop) == (32, 16)
    params = torch.zeros(sum(o * i for o, i in shapes), dtype=torch.float64)
    # first layer: unit weight only on padded column 31 -> hidden = 1 everywhere
    params[: width * nip].view(width, nip)[:, 31] = 1.0
    off = width * nip
    params[off:off + width * width].view(width, width)[:] = torch.eye(width)
    off += width * width
    params[off:off + nop * width].view(nop, width)[:, 0] = 2.0
    out = ref_tcnn.mlp_fwd(torch.zeros(5, n_in), params, n_in, n_out, width, 2)
    assert out.shape == (5, 4)
    assert torch.all(out == 2.0)
