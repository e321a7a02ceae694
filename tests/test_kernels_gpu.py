"""Parity of every HIP kernel against the oracle / the reference's golden vectors.

Tolerances (BASELINE north_star: 1e-4 relative fp32, bit-exact for sample indices):
  * sampler z / pts: bit-exact;
  * preprocessor: <= 2 ulp-ish (2e-7 abs on [-1,1]) — fp64 libm differences only;
  * exact-f32 kernels (hash grid, SH, MLP f32 MFMA, composite, loss, Adam): 1e-4 relative
    (checked as |a-b| <= 1e-4 * max|b| + small atol);
  * f16 kernels: compared with an oracle that rounds at the same points, 1e-2 relative.
"""

import ctypes

import numpy as np
import pytest
import torch

from oracle import ref_path, ref_tcnn
from tests.conftest import golden

pytestmark = pytest.mark.gpu


def close(a, b, rel=1e-4, atol=1e-7):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item() if a.numel() else 0.0
    tol = rel * b.abs().max().item() + atol
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


# ------------------------------------------------------------------ K1 / K2
@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_sampler_bit_exact_vs_reference(dev, tag):
    from atmonr_amd.samplers import sample_uniform_bins

    g = golden("sampler.npz")
    batch = {k: torch.from_numpy(g[f"{tag}_{n}"]).to(dev) for k, n in
             [("origin", "origin"), ("dir", "dir"), ("len", "len")]}
    u = torch.from_numpy(g[f"{tag}_u"]).to(dev)
    pts, z = sample_uniform_bins(batch, u.shape[1], u=u)
    assert torch.equal(z.cpu(), torch.from_numpy(g[f"{tag}_z"]))
    assert torch.equal(pts.cpu(), torch.from_numpy(g[f"{tag}_pts"]))
    pts, z = sample_uniform_bins(batch, u.shape[1], random=False)
    assert torch.equal(z.cpu(), torch.from_numpy(g[f"{tag}_z_mid"]))
    assert torch.equal(pts.cpu(), torch.from_numpy(g[f"{tag}_pts_mid"]))


def test_sampler_empty_batch(dev):
    from atmonr_amd.samplers import sample_uniform_bins

    b = {"origin": torch.zeros(0, 3, device=dev), "dir": torch.zeros(0, 3, device=dev),
         "len": torch.zeros(0, device=dev)}
    pts, z = sample_uniform_bins(b, 64)
    assert pts.shape == (0, 64, 3) and z.shape == (0, 64)


@pytest.mark.parametrize("B", [0, 1, 777, 8192])
def test_gather_rows_and_surface_input_bit_exact(dev, B):
    """anr_gather_rows == per-field torch indexing (harp2.py:392-420); the surface input
    kernel == the torch ops of instant_ngp.py:143,150,173, bit for bit."""
    from atmonr_amd import _lib

    g = torch.Generator().manual_seed(B)
    R = 10000
    srcs = [torch.randn(R, 3, generator=g), torch.randn(R, 3, generator=g),
            torch.randn(R, generator=g).double(), torch.rand(R, generator=g),
            torch.randint(0, 4, (R,), generator=g), torch.randn(R, 7, generator=g)]
    srcs = [s.to(dev).contiguous() for s in srcs]
    idx = torch.randint(0, R, (B,), generator=g).to(dev)
    outs = _lib.gather_rows(idx, srcs)
    for s, o in zip(srcs, outs):
        assert o.dtype == s.dtype and torch.equal(o, s[idx])
    o, d, ln = outs[0], outs[1], outs[3]
    out = torch.empty(B, 5, device=dev)
    _lib.call("anr_ingp_surface_input", _lib.ptr(o), _lib.ptr(d), _lib.ptr(ln), B,
              _lib.ptr(out), _lib.stream(dev))
    ps = (o + d * ln[:, None] + 1) / 2
    assert torch.equal(out, torch.cat([ps[:, :2], d], dim=1))


def _prep_from_golden(g, tag, remap=False, alt_compress=1.0):
    from atmonr_amd.datasets.synthetic import PointPreprocessor

    scale, lat_min, lat_range, lon_min, lon_range, h0, shift = g[f"{tag}_meta"].tolist()
    off = g[f"{tag}_offset"].tolist()
    pp = PointPreprocessor(scale, tuple(off), lat_min, lat_range, lon_min, lon_range, h0,
                           bool(shift))
    return pp, pp.params(ngp_remap=remap, alt_compress=alt_compress)


@pytest.mark.parametrize("tag", ["std", "dateline"])
def test_preprocessor_vs_reference(dev, tag):
    from atmonr_amd.samplers import preprocess_points, sample_and_preprocess

    g = golden("preprocess.npz")
    pp, prm = _prep_from_golden(g, tag)
    pts = torch.from_numpy(g[f"{tag}_pts"]).to(dev)
    out = preprocess_points(pts, prm).cpu().numpy()
    ref = g[f"{tag}_coords"]
    assert np.abs(out - ref).max() <= 2e-7
    assert (out == ref).mean() > 0.99
    # fused sampler + preprocessor + Instant-NGP remap == op-by-op reference path
    _, prm8 = _prep_from_golden(g, tag, remap=True, alt_compress=8.0)
    batch = {"origin": torch.from_numpy(g[f"{tag}_ray_origin"]).to(dev),
             "dir": torch.from_numpy(g[f"{tag}_ray_dir"]).to(dev),
             "len": torch.from_numpy(g[f"{tag}_ray_len"]).to(dev)}
    torch.manual_seed(7)
    u = torch.rand(batch["origin"].shape[0], 32, device=dev)
    _, z, coords = sample_and_preprocess(batch, 32, prm8, u=u)
    p_ref, z_ref = ref_path.sample_uniform_bins(*(batch[k].cpu() for k in ("origin", "dir", "len")),
                                                u.cpu(), 32)
    assert torch.equal(z.cpu(), z_ref)
    c_ref = torch.from_numpy(ref_path.preprocess_horizontal(
        p_ref.numpy(), pp.scale, pp.offset, pp.lat_min, pp.lat_range, pp.lon_min, pp.lon_range,
        pp.ray_origin_height, pp.shift_lon))
    c_ref = (c_ref + 1) / 2
    c_ref[..., 2] = c_ref[..., 2] / 8
    assert (coords.cpu() - c_ref).abs().max() <= 2e-7


# ------------------------------------------------------------------ K3 / K4
def _grid_inputs(dev, cfg, M, coherent, seed=0):
    gen = torch.Generator().manual_seed(seed)
    if coherent:  # ray-like: consecutive samples along straight lines
        R = -(-M // 256)
        o = torch.rand(R, 1, cfg[0], generator=gen)
        d = (torch.rand(R, 1, cfg[0], generator=gen) - 0.5) * 0.3
        t = torch.linspace(0, 1, 256)[None, :, None]
        x = (o + d * t).clamp(0, 1).reshape(-1, cfg[0])[:M]
    else:
        x = torch.rand(M, cfg[0], generator=gen)
    return x.contiguous()


# hash-grid kernel generations (anr_hashgrid_force_v1 modes): "default" = forward v6
# (branch-free corners, buffer addressing) with backward v2, "v1" = both v1 (the generic
# kernels), "v1fwd" = forward v1 walker with backward v2 (the r01 default), "rtstride" =
# the default with the backward's run-time-stride instantiation
_HASH_MODES = {"default": 0, "v1": 1, "v1fwd": 6, "rtstride": 7}


@pytest.fixture(params=["default", "v1", "v1fwd", "rtstride"])
def hash_path(request):
    from atmonr_amd import _lib

    prev = _lib.load().anr_hashgrid_force_v1(_HASH_MODES[request.param])
    yield request.param
    _lib.load().anr_hashgrid_force_v1(prev)


@pytest.mark.parametrize("cfg,M,coherent", [((3, 16, 16, 1.3819, 19), 5000, False),
                                            ((3, 16, 16, 1.3819, 19), 8192, True),
                                            ((3, 16, 16, 1.3819, 21), 3001, True),
                                            ((2, 16, 16, 1.3819, 19), 4096, False),
                                            ((3, 6, 4, 2.0, 10), 777, True),
                                            ((3, 16, 16, 1.3819, 19), 300000, True),
                                            ((2, 16, 16, 1.3819, 19), 70000, True),
                                            ((3, 20, 16, 1.3, 15), 2000, True)])
def test_hashgrid_fwd_bwd_f32(dev, hash_path, cfg, M, coherent):
    from atmonr_amd import _lib

    d = _lib.hashgrid_desc(cfg[0], cfg[1], 2, cfg[2], cfg[3], cfg[4])
    gen = torch.Generator().manual_seed(1)
    table = (torch.rand(d.n_params, generator=gen) * 2 - 1)
    x = _grid_inputs(dev, cfg, M, coherent)
    out = torch.empty(M, cfg[1] * 2, device=dev)
    s = _lib.stream(dev)
    td, xd = table.to(dev), x.to(dev)
    _lib.call("anr_hashgrid_fwd", ctypes.byref(d), xd.data_ptr(), cfg[0], M, td.data_ptr(),
              _lib.F32, out.data_ptr(), _lib.F32, out.stride(0), s)
    ref = ref_tcnn.hashgrid_fwd(x.numpy(), table.numpy(), cfg)
    close(out, ref, rel=1e-5)
    dout = torch.randn(M, cfg[1] * 2, generator=gen)
    dtab = torch.zeros(d.n_params, device=dev)
    dd = dout.to(dev)
    _lib.call("anr_hashgrid_bwd", ctypes.byref(d), xd.data_ptr(), cfg[0], M, dd.data_ptr(),
              _lib.F32, dd.stride(0), dtab.data_ptr(), s)
    gref = ref_tcnn.hashgrid_bwd(x.numpy(), dout.numpy(), cfg, d.n_params // 2)
    close(dtab, gref, rel=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", [0, 6])
def test_hashgrid_bench_size_adjoint_and_spot_rows(dev, mode):
    """Bench size (8192 rays x 1024 samples, the config-3 grid): the chunk lengths chosen
    only at this size (forward 128, backward 256 samples per chunk) against the oracle on
    4096 spot rows (forward), and the adjoint identity <g, fwd(t)> = <bwd(g), t> over all
    8.39 M samples (backward: a missed or doubled corner flush at a chunk end would break
    it by ~1e-3 of the scale; f32 rounding stays ~1e-7). f32 table and gradients."""
    from atmonr_amd import _lib

    cfg = (3, 16, 16, 1.3819, 19)
    B, N = 8192, 1024
    M = B * N
    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    gen = torch.Generator(device=dev).manual_seed(7)
    o = torch.rand(B, 1, 3, device=dev, generator=gen)
    dr = (torch.rand(B, 1, 3, device=dev, generator=gen) - 0.5) * 0.6
    t = torch.linspace(0, 1, N, device=dev)[None, :, None]
    x = (o + dr * t).clamp(0, 1).reshape(M, 3).contiguous()
    table = torch.rand(d.n_params, device=dev, generator=gen) * 2 - 1
    out = torch.empty(M, 32, device=dev)
    s = _lib.stream(dev)
    lib = _lib.load()
    prev = lib.anr_hashgrid_force_v1(mode)
    _lib.call("anr_hashgrid_fwd", ctypes.byref(d), x.data_ptr(), 3, M, table.data_ptr(),
              _lib.F32, out.data_ptr(), _lib.F32, out.stride(0), s)
    rows = torch.randint(0, M, (4096,), device=dev, generator=gen)
    ref = ref_tcnn.hashgrid_fwd(x[rows].cpu().numpy(), table.cpu().numpy(), cfg)
    close(out[rows], ref, rel=1e-5)
    g = torch.randn(M, 32, device=dev, generator=gen)
    dtab = torch.zeros(d.n_params, device=dev)
    _lib.call("anr_hashgrid_bwd", ctypes.byref(d), x.data_ptr(), 3, M, g.data_ptr(), _lib.F32,
              g.stride(0), dtab.data_ptr(), s)
    lib.anr_hashgrid_force_v1(prev)
    lhs = torch.dot(g.flatten().double(), out.flatten().double()).item()
    rhs = torch.dot(dtab.double(), table.double()).item()
    scale = torch.dot(g.flatten().double().abs(), out.flatten().double().abs()).item()
    assert abs(lhs - rhs) <= 1e-5 * scale, (lhs, rhs, scale)


@pytest.mark.parametrize("M,run", [(300000, 100), (70001, 37), (8192 * 16, 512)])
def test_hashgrid_bwd_zero_gradient_runs(dev, M, run):
    """The v2 backward skips batches whose dL/dy is zero in every lane (flushing the
    pending corner sums first): with runs of zero rows (the reference numerics' f16
    underflow) the table gradient still equals the oracle's."""
    from atmonr_amd import _lib

    cfg = (3, 16, 16, 1.3819, 19)
    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    x = _grid_inputs(dev, cfg, M, True, seed=11)
    gen = torch.Generator().manual_seed(12)
    dout = torch.randn(M, 32, generator=gen)
    zero = (torch.arange(M) // run) % 3 != 0  # two runs of zeros, then one of gradients
    dout[zero] = 0.0
    dtab = torch.zeros(d.n_params, device=dev)
    xd, dd = x.to(dev), dout.to(dev)
    _lib.call("anr_hashgrid_bwd", ctypes.byref(d), xd.data_ptr(), 3, M, dd.data_ptr(),
              _lib.F32, dd.stride(0), dtab.data_ptr(), _lib.stream(dev))
    gref = ref_tcnn.hashgrid_bwd(x.numpy(), dout.numpy(), cfg, d.n_params // 2)
    close(dtab, gref, rel=1e-5, atol=1e-5)


def test_hashgrid_bwd_request_count_instrument(dev):
    """anr_hashgrid_bwd_count_requests (bench.py's in-run request count): with every
    dL/denc nonzero it equals the CPU replay of the kernel's walk (tools/hash_requests.py,
    itself checked against rocprofv3 TCC_EA0_ATOMIC_sum: 2.5086 vs 2.508 per sample);
    all-zero gradients make no requests; zeroing the gradient of some samples can only
    remove requests (the zero-sum corners the kernel skips); the gradient buffer is not
    written. Ray-like coordinates at 64 rays x 1,024 samples (the PSNR test's shape)."""
    from atmonr_amd import _lib
    from tools import hash_requests

    cfg = (3, 16, 16, 1.3819, 19)
    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    M = 64 * 1024
    gen = torch.Generator(device=dev).manual_seed(5)
    # 64 straight rays of 1,024 samples inside the unit cube (no clamping: a sample exactly
    # on a cell face gives a corner a zero weight, a zero sum the kernel skips and the CPU
    # replay does not model)
    o = 0.2 + 0.6 * torch.rand(64, 1, 3, device=dev, generator=gen)
    dr = (torch.rand(64, 1, 3, device=dev, generator=gen) - 0.5) * 0.3
    x = (o + dr * torch.linspace(0, 1, 1024, device=dev)[None, :, None]).reshape(M, 3).contiguous()
    g = torch.randn(M, 32, device=dev, generator=gen)
    g[g == 0] = 1.0
    dtab = torch.zeros(d.n_params, device=dev)
    s = _lib.stream(dev)

    def count(grad):
        c = torch.zeros(1, dtype=torch.int64, device=dev)
        _lib.call("anr_hashgrid_bwd_count_requests", ctypes.byref(d), x.data_ptr(), 3, M,
                  grad.data_ptr(), _lib.F32, grad.stride(0), dtab.data_ptr(), c.data_ptr(), s)
        torch.cuda.synchronize()
        return int(c.item())

    full = count(g)
    replay = hash_requests.count(x, d)
    # the replay counts level by level; the instrument counts distinct segments over the
    # whole wave instruction, so two levels' corners in one segment at a table-region
    # border are one request there (and a rare sample exactly on a cell face gives a zero
    # sum): measured 580,240 vs 580,261 (3.6e-5)
    assert full <= replay and replay - full <= 1e-4 * replay, (full, replay)
    assert count(torch.zeros_like(g)) == 0
    gz = g.clone()
    gz[torch.rand(M, device=dev, generator=gen) < 0.7] = 0.0
    part = count(gz)
    assert 0 < part < full
    assert not dtab.any()


def test_hashgrid_f16_table_and_strided_output(dev, hash_path):
    from atmonr_amd import _lib

    cfg = (3, 16, 16, 1.3819, 19)
    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    gen = torch.Generator().manual_seed(2)
    table = ((torch.rand(d.n_params, generator=gen) * 2 - 1) * 1e-2).half()
    M = 4000
    x = _grid_inputs(dev, cfg, M, True, seed=3)
    big = torch.full((M, 40), -7.0, device=dev, dtype=torch.float16)  # write cols 4..35
    xd = x.to(dev)
    table_d = table.to(dev)  # keep the device copy alive across the launch
    _lib.call("anr_hashgrid_fwd", ctypes.byref(d), xd.data_ptr(), 3, M, table_d.data_ptr(),
              _lib.F16, big.data_ptr() + 4 * 2, _lib.F16, 40, _lib.stream(dev))
    ref = ref_tcnn.hashgrid_fwd(x.numpy(), table.float().numpy(), cfg)
    close(big[:, 4:36].float(), ref, rel=2e-3, atol=1e-5)
    assert torch.all(big[:, :4] == -7) and torch.all(big[:, 36:] == -7)


# ------------------------------------------------------------------ K5
@pytest.mark.parametrize("degree", [1, 2, 3, 4])
def test_sh_fwd_bwd(dev, degree):
    from atmonr_amd import _lib

    gen = torch.Generator().manual_seed(degree)
    M = 1000
    x = torch.rand(M, 3, generator=gen)
    out = torch.empty(M, degree * degree, device=dev)
    xd = x.to(dev)
    s = _lib.stream(dev)
    _lib.call("anr_sh_fwd", degree, xd.data_ptr(), 3, M, out.data_ptr(), _lib.F32,
              out.stride(0), s)
    close(out, ref_tcnn.sh(x.numpy(), degree), rel=1e-6, atol=1e-6)
    dout = torch.randn(M, degree * degree, generator=gen)
    dx = torch.zeros(M, 3, device=dev)
    dout_d = dout.to(dev)
    _lib.call("anr_sh_bwd", degree, xd.data_ptr(), 3, M, dout_d.data_ptr(), _lib.F32,
              degree * degree, dx.data_ptr(), 3, s)
    xx = x.double().requires_grad_(True)
    sh = torch.from_numpy(ref_tcnn.sh(x.numpy(), degree))  # value check only
    # autograd of the same polynomial in torch for the gradient
    X, Y, Z = (xx * 2 - 1).unbind(1)
    terms = [torch.full_like(X, 0.28209479177387814)]
    if degree > 1:
        c = 0.48860251190291987
        terms += [-c * Y, c * Z, -c * X]
    if degree > 2:
        terms += [1.0925484305920792 * X * Y, -1.0925484305920792 * Y * Z,
                  0.94617469575755997 * Z * Z - 0.31539156525251999,
                  -1.0925484305920792 * X * Z, 0.54627421529603959 * (X * X - Y * Y)]
    if degree > 3:
        terms += [0.59004358992664352 * Y * (-3.0 * X * X + Y * Y),
                  2.8906114426405538 * X * Y * Z, 0.45704579946446572 * Y * (1.0 - 5.0 * Z * Z),
                  0.3731763325901154 * Z * (5.0 * Z * Z - 3.0),
                  0.45704579946446572 * X * (1.0 - 5.0 * Z * Z),
                  1.4453057213202769 * Z * (X * X - Y * Y),
                  0.59004358992664352 * X * (-X * X + 3.0 * Y * Y)]
    tt = torch.stack(terms, 1)
    assert torch.allclose(tt.detach(), sh)
    if degree == 1:  # constant term: zero gradient
        assert torch.all(dx == 0)
        return
    (tt * dout.double()).sum().backward()
    close(dx, xx.grad, rel=1e-5, atol=1e-5)


# ------------------------------------------------------------------ K6 / K7
MLP_CASES = [(32, 16, 32, 1, False), (32, 16, 64, 1, False), (19, 4, 32, 2, True),
             (19, 4, 64, 2, False), (36, 4, 32, 2, False), (36, 4, 64, 2, True),
             (16, 3, 16, 3, False), (40, 20, 128, 1, True), (10, 16, 64, 2, False)]


@pytest.fixture(params=["specialised", "generic"])
def mlp_path(request):
    from atmonr_amd import _lib

    prev = _lib.load().anr_mlp_force_generic(1 if request.param == "generic" else 0)
    yield request.param
    _lib.load().anr_mlp_force_generic(prev)


@pytest.mark.parametrize("n_in,n_out,width,n_hidden,out_relu", MLP_CASES)
@pytest.mark.parametrize("half", [False, True])
def test_mlp_fwd_bwd(dev, mlp_path, n_in, n_out, width, n_hidden, out_relu, half):
    from atmonr_amd import _lib

    d = _lib.mlp_desc(n_in, n_out, width, n_hidden, out_relu)
    nparam = _lib.load().anr_mlp_n_params(ctypes.byref(d))
    gen = torch.Generator().manual_seed(width + n_in)
    params = torch.randn(nparam, generator=gen) * (1.0 / width) ** 0.5
    M = 1001  # not a multiple of the 16-row tile
    x = torch.randn(M, n_in, generator=gen)
    dt = torch.float16 if half else torch.float32
    prec = _lib.F16 if half else _lib.F32
    s = _lib.stream(dev)
    pd = params.to(dev).to(dt)
    xd = x.to(dev).to(dt)
    out = torch.empty(M, n_out, device=dev, dtype=torch.float32)
    _lib.call("anr_mlp_fwd", ctypes.byref(d), prec, pd.data_ptr(), xd.data_ptr(),
              _lib.dtype_code(dt), n_in, M, out.data_ptr(), _lib.F32, n_out, s)
    xr = x.double().requires_grad_(True)
    pr = params.double().requires_grad_(True)
    ref = ref_tcnn.mlp_fwd(xr, pr, n_in, n_out, width, n_hidden, out_relu, half=half)
    rel = 1e-2 if half else 1e-4
    close(out, ref.detach(), rel=rel, atol=1e-6)
    dout = torch.randn(M, n_out, generator=gen) * 1e-3
    ref.backward(dout.double())
    dparams = torch.zeros(nparam, device=dev)
    din = torch.empty(M, n_in, device=dev, dtype=torch.float32)
    dd = dout.to(dev)
    _lib.call("anr_mlp_bwd", ctypes.byref(d), prec, pd.data_ptr(), xd.data_ptr(),
              _lib.dtype_code(dt), n_in, M, dd.data_ptr(), _lib.F32, n_out, din.data_ptr(),
              _lib.F32, n_in, dparams.data_ptr(), s)
    close(din, xr.grad, rel=rel * 2, atol=1e-8)
    close(dparams, pr.grad, rel=rel * 2, atol=1e-8)


@pytest.mark.parametrize("n_in,n_out,width,n_hidden,out_relu", MLP_CASES)
@pytest.mark.parametrize("M", [8192, 1001, 16])
def test_mlp_bwd_workspace(dev, n_in, n_out, width, n_hidden, out_relu, M):
    """anr_mlp_bwd_ws: the slab path (per-wavefront dW rows, fixed-order sum) gives the
    atomics path's dparams (accumulated into, not overwritten), is bit-reproducible, and a
    too-small workspace falls back to the atomics."""
    from atmonr_amd import _lib

    lib = _lib.load()
    d = _lib.mlp_desc(n_in, n_out, width, n_hidden, out_relu)
    nparam = lib.anr_mlp_n_params(ctypes.byref(d))
    ws_bytes = lib.anr_mlp_bwd_workspace_bytes(ctypes.byref(d), M)
    specialised = n_out <= 16 and width in (32, 64) and n_hidden in (1, 2)
    assert (ws_bytes > 0) == specialised and ws_bytes % 4 == 0
    if not specialised:  # generic kernel: atomics only, no workspace
        return
    gen = torch.Generator().manual_seed(M + width)
    pd = (torch.randn(nparam, generator=gen) * (1.0 / width) ** 0.5).to(dev).half()
    xd = torch.randn(M, n_in, generator=gen).to(dev).half()
    dd = (torch.randn(M, n_out, generator=gen) * 1e-3).to(dev)
    base = torch.randn(nparam, generator=gen).to(dev) * 1e-3
    s = _lib.stream(dev)

    def run(ws, nbytes):
        dp = base.clone()
        din = torch.empty(M, n_in, device=dev)
        _lib.call("anr_mlp_bwd_ws", ctypes.byref(d), _lib.F16, pd.data_ptr(), xd.data_ptr(),
                  _lib.F16, n_in, M, dd.data_ptr(), _lib.F32, n_out, din.data_ptr(), _lib.F32,
                  n_in, dp.data_ptr(), _lib.ptr(ws), nbytes, s)
        return dp, din

    ws = torch.full((ws_bytes // 4,), float("nan"), device=dev)  # every slot is written
    dp_a, din_a = run(None, 0)
    dp_s, din_s = run(ws, ws_bytes)
    dp_s2, _ = run(ws, ws_bytes)
    dp_small, _ = run(ws, 4 * nparam - 4)
    assert torch.equal(din_a, din_s)
    assert torch.equal(dp_s, dp_s2)
    g = dp_a - base
    assert ((dp_s - base - g).norm() / g.norm()).item() <= 1e-5
    assert ((dp_small - base - g).norm() / g.norm()).item() <= 1e-5
    assert lib.anr_mlp_bwd_workspace_bytes(ctypes.byref(d), 1 << 20) == 0


# ------------------------------------------------------------------ K8
@pytest.fixture(params=["blocked", "generic"])
def comp_path(request):
    from atmonr_amd import _lib

    prev = _lib.load().anr_composite_force_generic(1 if request.param == "generic" else 0)
    yield request.param
    _lib.load().anr_composite_force_generic(prev)


@pytest.mark.parametrize("tag", ["f32", "f32long", "f32multi", "f16"])
def test_composite_vs_reference(dev, comp_path, tag):
    from atmonr_amd.graphics_utils import render, render_with_surface

    g = golden("render.npz")
    dt = torch.float16 if tag == "f16" else torch.float32
    t = {k: torch.from_numpy(g[f"{tag}_{k}"]) for k in
         ("z", "color", "sigma", "cs", "gcm", "gatmo", "gsurf", "gw")}
    z = t["z"].to(dev).requires_grad_(True)
    c = t["color"].to(dev).to(dt).requires_grad_(True)
    s = t["sigma"].to(dev).to(dt).requires_grad_(True)
    cs = t["cs"].to(dev).to(dt).requires_grad_(True)
    cm, alpha, w, atmo, surf = render_with_surface(z, c, s, cs)
    rel = 1e-4 if dt == torch.float32 else 2e-2
    atol = 1e-6 if dt == torch.float32 else 2e-2
    for name, out in [("cm", cm), ("alpha", alpha), ("w", w), ("atmo", atmo), ("surf", surf)]:
        close(out.float(), torch.from_numpy(g[f"{tag}_{name}"]), rel=rel, atol=atol)
    loss = ((cm.float() * t["gcm"].to(dev).float()).sum() + (atmo.float() * t["gatmo"].to(dev)).sum()
            + (surf.float() * t["gsurf"].to(dev)).sum() + (w.float() * t["gw"].to(dev)).sum())
    loss.backward()
    if dt == torch.float32:
        for name, ten in [("dcolor", c), ("dsigma", s), ("dcs", cs), ("dz", z)]:
            close(ten.grad.float(), torch.from_numpy(g[f"{tag}_{name}"]), rel=1e-4, atol=1e-5)
    cm2, _, w2 = render(t["z"].to(dev), t["color"].to(dev).to(dt), t["sigma"].to(dev).to(dt))
    close(cm2.float(), torch.from_numpy(g[f"{tag}_plain_cm"]), rel=rel, atol=atol)


@pytest.mark.parametrize("N,S", [(300, 1), (700, 4), (2000, 1), (1024, 4), (200, 4)])
def test_composite_long_rays_vs_oracle(dev, N, S):
    """Register-blocked paths at lengths with partial last lanes: one wave per ray up to 256
    samples, one 4-wave block per ray above (cross-wave scans through LDS)."""
    from atmonr_amd.graphics_utils import render_with_surface

    gen = torch.Generator().manual_seed(N + S)
    B = 5
    z = torch.sort(torch.rand(B, N, generator=gen), dim=1).values * 20
    color = torch.rand(B, N, 4, generator=gen) * 2
    sigma = torch.rand(B, N, S, generator=gen) * (30.0 / N)
    cs = torch.rand(B, 4, generator=gen)
    ins = [t.clone().requires_grad_(True) for t in (z, color, sigma, cs)]
    ref = ref_path.render_with_surface(*ins)
    gouts = [torch.randn(r.shape, generator=gen) for r in ref]
    sum((r * g).sum() for r, g in zip(ref, gouts)).backward()
    dins = [t.to(dev).requires_grad_(True) for t in (z, color, sigma, cs)]
    out = render_with_surface(*dins)
    for o, r in zip(out, ref):
        close(o, r.detach(), rel=1e-4, atol=1e-6)
    sum((o * g.to(dev)).sum() for o, g in zip(out, gouts)).backward()
    for d, r in zip(dins, ins):
        close(d.grad, r.grad, rel=1e-4, atol=1e-5)


def test_composite_known_answers(dev, comp_path):
    from atmonr_amd.graphics_utils import render_with_surface

    B, N = 3, 100
    z = torch.linspace(0, 10, N, device=dev)[None].expand(B, N).contiguous()
    color = torch.rand(B, N, 4, device=dev)
    cs = torch.rand(B, 4, device=dev)
    # zero density: C = C_surf exactly
    cm, _, w, atmo, surf = render_with_surface(z, color, torch.zeros(B, N, 1, device=dev), cs)
    assert torch.all(w == 0) and torch.all(atmo == 0)
    assert torch.equal(cm, cs)
    # uniform density sigma: transmittance to the surface is exp(-sigma * z_end)
    sig = 0.07
    cm, _, w, atmo, surf = render_with_surface(z, torch.ones_like(color),
                                               torch.full((B, N, 1), sig, device=dev), cs)
    T = torch.exp(torch.tensor(-sig * 10.0))
    close(surf, (T * cs.cpu()), rel=1e-5)
    close(atmo, torch.full((B, 4), 1 - T.item()), rel=1e-5)


# ------------------------------------------------------------------ K9
@pytest.mark.parametrize("name", ["dark", "hdr", "l1", "l1_plus_hdr", "mse", "mse_plus_hdr"])
def test_losses_vs_reference(dev, name):
    from atmonr_amd import losses

    g = golden("losses.npz")
    p = torch.from_numpy(g["pred"]).to(dev).requires_grad_(True)
    val = losses.LOSSES[name](p, torch.from_numpy(g["gt"]).to(dev), float(g["max_i"]))
    val.backward()
    close(val.detach(), torch.tensor(g[f"{name}_val"]), rel=1e-5)
    close(p.grad, torch.from_numpy(g[f"{name}_grad"]), rel=1e-4, atol=1e-9)


def test_indexed_loss_matches_take_along_dim(dev):
    from atmonr_amd.losses import indexed_loss

    gen = torch.Generator().manual_seed(5)
    B = 3000
    cm = (torch.rand(B, 4, generator=gen) * 20).to(dev).requires_grad_(True)
    idx = torch.randint(0, 4, (B,), generator=gen).to(dev)
    gt = (torch.rand(B, generator=gen) * 20).to(dev)
    val = indexed_loss("mse_plus_hdr", cm, idx, gt, 25.0)
    val.backward()
    cr = cm.detach().cpu().double().requires_grad_(True)
    pr = torch.take_along_dim(cr, idx.cpu()[:, None], 1)[:, 0]
    ref = ref_path.LOSSES["mse_plus_hdr"](pr, gt.cpu().double(), 25.0)
    ref.backward()
    close(val.detach(), ref.detach(), rel=1e-5)
    close(cm.grad, cr.grad, rel=1e-4, atol=1e-10)


# ------------------------------------------------------------------ K10
@pytest.mark.parametrize("decoupled,wd", [(True, 1e-2), (True, 0.0), (False, 1e-3)])
def test_adam_matches_torch(dev, decoupled, wd):
    from atmonr_amd.optim import FusedAdam

    gen = torch.Generator().manual_seed(9)
    p0 = torch.randn(10007, generator=gen)
    grads = [torch.randn(10007, generator=gen) * 0.1 for _ in range(5)]
    pa = torch.nn.Parameter(p0.clone().to(dev))
    pb = torch.nn.Parameter(p0.clone())
    kw = dict(lr=1e-2, betas=(0.9, 0.99), eps=1e-15, weight_decay=wd)
    oa = FusedAdam([pa], decoupled=decoupled, **kw)
    ob = (torch.optim.AdamW if decoupled else torch.optim.Adam)([pb], foreach=False, **kw)
    for gr in grads:
        pa.grad = gr.to(dev)
        pb.grad = gr.clone()
        oa.step()
        ob.step()
    close(pa.detach(), pb.detach(), rel=1e-5, atol=1e-6)
    close(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"], rel=1e-5, atol=1e-12)


@pytest.mark.parametrize("decoupled", [True, False])
def test_adam_multi_tensor_matches_torch_and_per_tensor(dev, decoupled):
    """anr_adam_step_multi (FusedAdam's default): 19 tensors (more than one launch's 16,
    one of them empty), two param groups with their own lr / weight decay, against
    torch.optim.AdamW / Adam, and bit for bit against the per-tensor launches."""
    from atmonr_amd.optim import FusedAdam

    gen = torch.Generator().manual_seed(3)
    sizes = [1, 1023, 1024, 1025, 4097, 0, 77777] + [300 + 17 * i for i in range(12)]
    p0 = [torch.randn(n, generator=gen) for n in sizes]
    grads = [[torch.randn(n, generator=gen) * 0.1 for n in sizes] for _ in range(4)]

    def groups(ps):
        return [{"params": ps[:9], "weight_decay": 0.0, "lr": 1e-2},
                {"params": ps[9:], "weight_decay": 1e-2, "lr": 3e-3}]

    kw = dict(betas=(0.9, 0.99), eps=1e-15)
    pa = [torch.nn.Parameter(x.clone().to(dev)) for x in p0]
    pc = [torch.nn.Parameter(x.clone().to(dev)) for x in p0]
    pb = [torch.nn.Parameter(x.clone()) for x in p0]
    oa = FusedAdam(groups(pa), decoupled=decoupled, **kw)
    oc = FusedAdam(groups(pc), decoupled=decoupled, **kw)
    oc.multi_tensor = False
    ob = (torch.optim.AdamW if decoupled else torch.optim.Adam)(groups(pb), foreach=False, **kw)
    for gr in grads:
        for x, y, z, g in zip(pa, pc, pb, gr):
            x.grad, y.grad, z.grad = g.to(dev), g.to(dev), g.clone()
        oa.step()
        oc.step()
        ob.step()
    for x, y, z in zip(pa, pc, pb):
        assert torch.equal(x.detach(), y.detach())
        if z.numel():
            close(x.detach(), z.detach(), rel=1e-5, atol=1e-6)
    for x, z in zip(pa, pb):
        if z.numel():
            close(oa.state[x]["exp_avg_sq"], ob.state[z]["exp_avg_sq"], rel=1e-5, atol=1e-12)


@pytest.mark.parametrize("multi", [True, False])
def test_adam_groups_with_their_own_betas_eps(dev, multi):
    """Param groups with different betas / eps each step with their own (as torch does):
    one multi-tensor launch per (betas, eps) group."""
    from atmonr_amd.optim import FusedAdam

    gen = torch.Generator().manual_seed(5)
    p0 = [torch.randn(n, generator=gen) for n in (513, 2049, 77)]
    grads = [[torch.randn(x.numel(), generator=gen) * 0.1 for x in p0] for _ in range(3)]

    def groups(ps):
        return [{"params": ps[:1], "betas": (0.9, 0.99), "eps": 1e-15},
                {"params": ps[1:2], "betas": (0.8, 0.9), "eps": 1e-8, "lr": 3e-3},
                {"params": ps[2:], "betas": (0.95, 0.999), "eps": 1e-6, "weight_decay": 0.1}]

    pa = [torch.nn.Parameter(x.clone().to(dev)) for x in p0]
    pb = [torch.nn.Parameter(x.clone()) for x in p0]
    oa = FusedAdam(groups(pa), lr=1e-2)
    oa.multi_tensor = multi
    ob = torch.optim.AdamW(groups(pb), lr=1e-2, foreach=False)
    for gr in grads:
        for x, z, g in zip(pa, pb, gr):
            x.grad, z.grad = g.to(dev), g.clone()
        oa.step()
        ob.step()
    for x, z in zip(pa, pb):
        close(x.detach(), z.detach(), rel=1e-5, atol=1e-6)


def test_adam_multi_validates_every_tensor_before_launching(dev):
    """A bad descriptor after the first 16 tensors leaves every parameter untouched."""
    import ctypes

    from atmonr_amd import _lib

    ps = [torch.randn(64, device=dev) for _ in range(18)]
    before = [p.clone() for p in ps]
    st = [(torch.randn(64, device=dev), torch.zeros(64, device=dev), torch.zeros(64, device=dev))
          for _ in ps]
    ts = [_lib.AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), None, 64,
                          1e-2, 0.0, 1) for p, (g, m, v) in zip(ps, st)]
    ts[17].grad = None  # null gradient pointer in the second launch's batch
    arr = (_lib.AdamTensor * len(ts))(*ts)
    with pytest.raises(_lib.ANRError, match="tensor 17"):
        _lib.call("anr_adam_step_multi", ctypes.addressof(arr), len(ts), 0.9, 0.99, 1e-15, 1, 0,
                  _lib.stream(dev))
    torch.cuda.synchronize()
    for p, b in zip(ps, before):
        assert torch.equal(p, b)


# ------------------------------------------------------------------ fused dir encoding + MLP
@pytest.mark.parametrize("width,half", [(64, True), (64, False), (32, True)])
def test_ingp_dir_mlp_matches_unfused(dev, width, half):
    """anr_ingp_dir_mlp_{fwd,bwd} == SH2(dir) | pos_out[:,1:] -> padded MLP (oracle)."""
    from atmonr_amd import _lib

    gen = torch.Generator().manual_seed(width)
    n_per_ray, R = 37, 29
    M = n_per_ray * R
    d = _lib.mlp_desc(19, 4, width, 2, True)
    nparam = _lib.load().anr_mlp_n_params(ctypes.byref(d))
    params = torch.randn(nparam, generator=gen) * (1.0 / width) ** 0.5
    pos_out = torch.randn(M, 16, generator=gen)
    dirs = torch.nn.functional.normalize(torch.randn(R, 3, generator=gen), dim=1)
    sh = torch.from_numpy(ref_tcnn.sh(dirs.repeat_interleave(n_per_ray, 0).numpy(), 2))
    # re-draw rows whose hidden pre-activations sit on a ReLU kink (|h| < 1e-4): there an
    # f32 kernel and the f64 reference legitimately disagree on the mask (seed 64 has a
    # row at 2e-8)
    w_in = params[: width * 32].double().view(width, 32)
    w_h = params[width * 32: width * 32 + width * width].double().view(width, width)
    for _ in range(20):
        x0 = torch.cat([sh, pos_out[:, 1:].double(), torch.ones(M, 13, dtype=torch.float64)], 1)
        h0 = x0 @ w_in.T
        h1 = torch.relu(h0) @ w_h.T
        tied = (torch.minimum(h0.abs().min(1).values, h1.abs().min(1).values) < 1e-4)
        if not tied.any():
            break
        pos_out[tied] = torch.randn(int(tied.sum()), 16, generator=gen)
    assert not tied.any()
    dt = torch.float16 if half else torch.float32
    prec = _lib.F16 if half else _lib.F32
    s = _lib.stream(dev)
    pd, pod, dd = params.to(dev).to(dt), pos_out.to(dev), dirs.to(dev)
    color = torch.empty(M, 4, device=dev)
    _lib.call("anr_ingp_dir_mlp_fwd", ctypes.byref(d), prec, pd.data_ptr(), pod.data_ptr(), 16,
              dd.data_ptr(), n_per_ray, M, color.data_ptr(), _lib.F32, 4, s)
    por = pos_out.double().requires_grad_(True)
    x = torch.cat([sh, por[:, 1:]], dim=1)
    pr = params.double().requires_grad_(True)
    ref = ref_tcnn.mlp_fwd(x, pr, 19, 4, width, 2, output_relu=True, half=half)
    rel = 1e-2 if half else 1e-4
    close(color, ref.detach(), rel=rel, atol=1e-6)
    dcol = torch.randn(M, 4, generator=gen) * 1e-2
    dsig = torch.randn(M, generator=gen) * 1e-2
    sig = torch.relu(por[:, 0])
    (ref * dcol.double()).sum().backward(retain_graph=True)
    (sig * dsig.double()).sum().backward()
    dpos = torch.empty(M, 16, device=dev)
    dparams = torch.zeros(nparam, device=dev)
    # device copies bound to names: a temporary's block would be reused by the next .to()
    dcol_d, dsig_d = dcol.to(dev), dsig.to(dev)
    _lib.call("anr_ingp_dir_mlp_bwd", ctypes.byref(d), prec, pd.data_ptr(), pod.data_ptr(), 16,
              dd.data_ptr(), n_per_ray, M, dcol_d.data_ptr(), 4, dsig_d.data_ptr(),
              dpos.data_ptr(), 16, dparams.data_ptr(), s)
    close(dpos, por.grad, rel=rel * 2, atol=1e-8)
    close(dparams, pr.grad, rel=rel * 2, atol=1e-8)


def _field_ref(enc, dirs, n_per_ray, pp, pd, width, nhd, nb, half=True):
    """sigma, color of instant_ngp.py:163-184 in float64 with the kernel's roundings
    (half=True: f16; half="bf16": bf16 operands)."""
    pos_out = ref_tcnn.mlp_fwd(enc, pp, 32, 16, width, 1, half=half)
    sh = torch.from_numpy(ref_tcnn.sh(dirs.detach().repeat_interleave(n_per_ray, 0).numpy(), 2))
    x = torch.cat([sh, pos_out[:, 1:]], dim=1)
    color = ref_tcnn.mlp_fwd(x, pd, 19, nb, width, nhd, output_relu=True, half=half)
    return torch.relu(pos_out[:, 0]), color, pos_out, x


def _field_preacts(enc, dirs, n_per_ray, pp, pd, width, nhd, half=True):
    """min |pre-activation| per row over every ReLU of the field (tie detector)."""
    h = ref_tcnn.rounder(half)
    P0 = h(pp[: 32 * width]).view(width, 32)
    P1 = h(pp[32 * width:]).view(16, width)
    a0 = h(enc) @ P0.T
    pos_out = h(torch.relu(a0)) @ P1.T
    sh = torch.from_numpy(ref_tcnn.sh(dirs.repeat_interleave(n_per_ray, 0).numpy(), 2))
    x = torch.cat([h(sh), h(pos_out[:, 1:]), torch.ones(enc.shape[0], 13, dtype=torch.float64)], 1)
    off, mins, hcur = 0, [a0.abs().min(1).values, pos_out[:, 0].abs()], x
    dims = [32] + [width] * nhd + [16]
    for k in range(nhd + 1):
        Wk = h(pd[off: off + dims[k + 1] * dims[k]]).view(dims[k + 1], dims[k])
        off += dims[k + 1] * dims[k]
        a = hcur @ Wk.T
        mins.append(a.abs().min(1).values if k < nhd else a[:, :4].abs().min(1).values)
        hcur = h(torch.relu(a))
    return torch.stack(mins, 1).min(1).values


@pytest.mark.gpu
@pytest.mark.parametrize("mma", ["f16", "bf16"])
@pytest.mark.parametrize("width,nhd,R", [(64, 2, 29), (64, 2, 300), (32, 2, 29), (64, 1, 29),
                                         (32, 1, 31)])
def test_ingp_field_matches_oracle(dev, width, nhd, R, mma):
    """anr_ingp_field_{pack,fwd,bwd} == pos MLP -> SH2|pos_out[:,1:] -> dir MLP (oracle),
    with the oracle rounding operands where the kernel does: f16 (the reference's tcnn
    precision) or bf16 (BASELINE configs[4]). Tolerances (relative to the largest value):
    f16 1e-2 forward, 2e-2 gradients; bf16 (8 significant bits, gradient tiles unscaled
    in bf16) 2e-2 forward, 5e-2 gradients."""
    from atmonr_amd import _lib

    half = "bf16" if mma == "bf16" else True
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    rf, rb = (2e-2, 5e-2) if mma == "bf16" else (1e-2, 2e-2)

    nb, n_per_ray = 4, 37
    M = n_per_ray * R
    gen = torch.Generator().manual_seed(1000 * width + 10 * nhd + R)
    pdsc = _lib.mlp_desc(32, 16, width, 1, False)
    ddsc = _lib.mlp_desc(19, nb, width, nhd, False)
    lib = _lib.load()
    assert lib.anr_ingp_field_supported(ctypes.byref(pdsc), ctypes.byref(ddsc)) == 1
    n_pp = lib.anr_mlp_n_params(ctypes.byref(pdsc))
    n_pd = lib.anr_mlp_n_params(ctypes.byref(ddsc))
    pp = torch.randn(n_pp, generator=gen) * (2.0 / 32) ** 0.5
    pd = torch.randn(n_pd, generator=gen) * (2.0 / width) ** 0.5
    enc = torch.rand(M, 32, generator=gen) * 2 - 1
    dirs = torch.nn.functional.normalize(torch.randn(R, 3, generator=gen), dim=1)
    for _ in range(40):  # keep every ReLU input away from 0 (f16 kernel vs f64 oracle)
        tied = _field_preacts(enc, dirs, n_per_ray, pp, pd, width, nhd, half) < 2e-3
        if not tied.any():
            break
        enc[tied] = torch.rand(int(tied.sum()), 32, generator=gen) * 2 - 1
    assert not tied.any()
    enc_h = enc.half()
    s = _lib.stream(dev)
    pp_d, pd_d, enc_d, dirs_d = pp.to(dev), pd.to(dev), enc_h.to(dev), dirs.to(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(ctypes.byref(pdsc), ctypes.byref(ddsc)),
                         device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", ctypes.byref(pdsc), ctypes.byref(ddsc), code,
              pp_d.data_ptr(), pd_d.data_ptr(), packed.data_ptr(), s)
    sigma = torch.empty(M, device=dev)
    color = torch.empty(M, nb, device=dev)
    _lib.call("anr_ingp_field_fwd", ctypes.byref(pdsc), ctypes.byref(ddsc), code,
              packed.data_ptr(), enc_d.data_ptr(), 32, dirs_d.data_ptr(), n_per_ray, M,
              sigma.data_ptr(), color.data_ptr(), nb, s)
    e64 = enc_h.double().requires_grad_(True)
    pr_p = pp.double().requires_grad_(True)
    pr_d = pd.double().requires_grad_(True)
    rs, rc, _, _ = _field_ref(e64, dirs, n_per_ray, pr_p, pr_d, width, nhd, nb, half)
    close(sigma, rs.detach(), rel=rf, atol=1e-4)
    close(color, rc.detach(), rel=rf, atol=1e-4)

    dcol = torch.randn(M, nb, generator=gen) * 1e-2
    dsig = torch.randn(M, generator=gen) * 1e-3
    ((rc * dcol.double()).sum() + (rs * dsig.double()).sum()).backward()
    dcol_d, dsig_d = dcol.to(dev), dsig.to(dev)
    d_enc = torch.full((M, 32), float("nan"), device=dev)
    g_pos = torch.full((n_pp,), 0.5, device=dev)  # accumulated into
    g_dir = torch.full((n_pd,), -0.25, device=dev)
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(ctypes.byref(pdsc), ctypes.byref(ddsc),
                                                      code, M)
    assert (ws_bytes == 0) == (mma == "bf16")
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    _lib.call("anr_ingp_field_bwd", ctypes.byref(pdsc), ctypes.byref(ddsc), code,
              packed.data_ptr(), enc_d.data_ptr(), 32, dirs_d.data_ptr(), n_per_ray, M,
              dsig_d.data_ptr(), dcol_d.data_ptr(), nb, d_enc.data_ptr(), 32, g_pos.data_ptr(),
              g_dir.data_ptr(), ws.data_ptr() if ws_bytes else None, ws_bytes, s)
    close(d_enc, e64.grad, rel=rb, atol=1e-7)
    close(g_pos - 0.5, pr_p.grad, rel=rb, atol=1e-7)
    close(g_dir + 0.25, pr_d.grad, rel=rb, atol=1e-7)
    if mma == "f16":  # a workspace below the queried size is refused, not overrun
        rc = lib.anr_ingp_field_bwd(ctypes.byref(pdsc), ctypes.byref(ddsc), code,
                                    packed.data_ptr(), enc_d.data_ptr(), 32, dirs_d.data_ptr(),
                                    n_per_ray, M, dsig_d.data_ptr(), dcol_d.data_ptr(), nb,
                                    d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(),
                                    ws.data_ptr(), ws_bytes - 4, s)
        assert rc == -1 and b"workspace" in lib.anr_last_error()


@pytest.mark.gpu
def test_ingp_field_unsupported_and_empty(dev):
    from atmonr_amd import _lib

    lib = _lib.load()
    pdsc = _lib.mlp_desc(32, 16, 64, 1, False)
    assert lib.anr_ingp_field_supported(ctypes.byref(pdsc),
                                        ctypes.byref(_lib.mlp_desc(19, 4, 64, 3, False))) == 0
    assert lib.anr_ingp_field_supported(ctypes.byref(_lib.mlp_desc(24, 16, 64, 1, False)),
                                        ctypes.byref(_lib.mlp_desc(19, 4, 64, 2, False))) == 0
    ddsc = _lib.mlp_desc(19, 4, 64, 2, False)
    rc = lib.anr_ingp_field_fwd(ctypes.byref(pdsc), ctypes.byref(_lib.mlp_desc(19, 4, 64, 3, False)),
                                _lib.F16, None, None, 32, None, 1, 10, None, None, 4, None)
    assert rc == -1 and b"unsupported" in lib.anr_last_error()
    rc = lib.anr_ingp_field_fwd(ctypes.byref(pdsc), ctypes.byref(ddsc), _lib.F32, None, None, 32,
                                None, 1, 10, None, None, 4, None)
    assert rc == -1 and b"mma_dtype" in lib.anr_last_error()
    assert lib.anr_ingp_field_fwd(ctypes.byref(pdsc), ctypes.byref(ddsc), _lib.F16, None, None,
                                  32, None, 1, 0, None, None, 4, None) == 0


@pytest.mark.parametrize("mma", ["f16", "bf16"])
@pytest.mark.parametrize("width,nhd,M", [(64, 2, 2654208), (64, 2, 77), (32, 1, 1000)])
def test_ingp_field_density_equals_field_sigma(dev, width, nhd, M, mma):
    """anr_ingp_field_density (the pos MLP only: extract / occupancy) returns exactly the
    full field forward's sigma, at the extract batch (32,768 columns x 81 altitudes) and
    ragged sizes."""
    from atmonr_amd import _lib

    nb = 4
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    g = torch.Generator(device=dev).manual_seed(width + M)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dirs = torch.full((1, 3), 0.5, device=dev)
    sig_full = torch.full((M,), -1.0, device=dev)
    color = torch.empty(M, nb, device=dev)
    _lib.call("anr_ingp_field_fwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
              dirs.data_ptr(), M, M, sig_full.data_ptr(), color.data_ptr(), nb, s)
    sig = torch.full((M + 1,), -1.0, device=dev)
    _lib.call("anr_ingp_field_density", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32, M,
              sig.data_ptr(), s)
    assert torch.equal(sig[:M], sig_full)
    assert sig[M].item() == -1.0 and (sig_full > 0).any()


@pytest.mark.parametrize("mma", ["f16", "bf16"])
@pytest.mark.parametrize("width,nhd", [(64, 2), (64, 1), (32, 2), (32, 1)])
def test_ingp_field_bwd_relaunch_deterministic(dev, width, nhd, mma):
    """Guard for the field backward's hand-placed hazard wait states (inline-asm MFMAs and
    ReLU masks): 12 launches on the same inputs give bit-identical dL/denc and parameter
    gradients equal up to the atomic flush order (2e-5 of the largest: f32 sums of ~16 K
    contributions in launch-dependent order; measured 1.0e-6). A missing wait
    state shows as launch-to-launch differences first (r03: the ReLU-mask asm fed MFMA
    operands without its two wait states, and the W=32 two-hidden-layer dir weight
    gradients differed from launch to launch by up to 3x their size). The static check
    of the same wait states is tests/test_mfma_hazards.py."""
    from atmonr_amd import _lib

    nb, R, n_per_ray = 4, 64, 256
    M = R * n_per_ray + 29
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    g = torch.Generator(device=dev).manual_seed(width + nhd)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.rand(R + 1, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dcol = torch.randn(M, nb, device=dev, generator=g) * 1e-2
    dsig = torch.randn(M, device=dev, generator=g) * 1e-3
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, code, M)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    first = None
    for _ in range(12):
        d_enc = torch.empty(M, 32, device=dev)
        g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
        _lib.call("anr_ingp_field_bwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
                  dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                  d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(),
                  ws.data_ptr() if ws_bytes else None, ws_bytes, s)
        if first is None:
            first = (d_enc, g_pos, g_dir)
            continue
        assert torch.equal(d_enc, first[0])
        for a, b in ((g_pos, first[1]), (g_dir, first[2])):
            assert (a - b).abs().max().item() <= 2e-5 * b.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("mma", ["f16", "bf16"])
@pytest.mark.parametrize("n_per_ray,R,extra,width,nhd", [
    (16, 37, 0, 64, 2),     # one ray per tile, every tile full
    (64, 29, 5, 64, 2),     # partial last tile (general tail loop)
    (1024, 3, 0, 64, 2),    # the bench's samples per ray
    (48, 11, 7, 32, 1),     # other network shapes
    (40, 13, 0, 64, 2),     # 40 % 16 != 0: the launcher keeps the general form
])
def test_field_fwd_uniform_tile_matches_general(mma, n_per_ray, R, extra, width, nhd):
    """The uniform-tile forward (scalar direction per 16-row tile, branch-free buffer stores;
    anr_ingp_field_force_fwd(1), the default) is bit-identical to the general form (0)."""
    from atmonr_amd import _lib

    dev = torch.device("cuda:0")
    M = R * n_per_ray + extra
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    g = torch.Generator(device=dev).manual_seed(5)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, 4, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.rand(R + 1, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    out = {}
    for mode in (0, 1):
        prev = lib.anr_ingp_field_force_fwd(mode)
        try:
            sigma = torch.full((M + 16,), float("nan"), device=dev)
            color = torch.full((M + 16, 4), float("nan"), device=dev)
            _lib.call("anr_ingp_field_fwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
                      dirs.data_ptr(), n_per_ray, M, sigma.data_ptr(), color.data_ptr(), 4, s)
            torch.cuda.synchronize(dev)
        finally:
            lib.anr_ingp_field_force_fwd(prev)
        out[mode] = (sigma, color)
    for a, b in zip(out[0], out[1]):
        assert torch.isfinite(a[:M]).all()
        assert torch.equal(a[:M], b[:M])
        assert torch.isnan(a[M:]).all() and torch.isnan(b[M:]).all()  # nothing past row M


def _field_torch_f32(enc_h, dirs, n_per_ray, pp, pd, width, nhd, nb, h):
    """The fused field in torch f32 on the device with the kernel's 16-bit roundings (h):
    pos 32 -> W -> 16, SH2 | pos_out[1:16] | 1.0 padding, dir 32 -> W (x nhd) -> 16 -> nb."""
    P0 = h(pp[: 32 * width]).view(width, 32)
    P1 = h(pp[32 * width:]).view(16, width)
    po = h(torch.relu(h(enc_h.float()) @ P0.T)) @ P1.T
    d = dirs.repeat_interleave(n_per_ray, 0) * 2 - 1
    c1 = 0.48860251190291987
    sh = torch.stack([torch.full_like(d[:, 0], 0.28209479177387814), -c1 * d[:, 1],
                      c1 * d[:, 2], -c1 * d[:, 0]], 1)
    x = torch.cat([h(sh), h(po[:, 1:]), torch.ones(po.shape[0], 13, device=po.device)], 1)
    dims, off = [32] + [width] * nhd + [16], 0
    for k in range(nhd + 1):
        Wk = h(pd[off: off + dims[k + 1] * dims[k]]).view(dims[k + 1], dims[k])
        off += dims[k + 1] * dims[k]
        x = x @ Wk.T
        if k < nhd:
            x = h(torch.relu(x))
    return torch.relu(po[:, 0]), torch.relu(x[:, :nb])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mma", ["f16", "bf16"])
def test_ingp_field_bench_size(dev, mma):
    """Fused field at the bench size (8192 rays x 1024 samples, width 64, 2 dir layers)
    against the same network in torch f32 on the device with the kernel's 16-bit
    roundings (autograd for the gradients), plus 2,048 spot rows against the f64 CPU
    oracle. Tolerances (of the largest value): sigma / color 2e-2 (f16) / 4e-2 (bf16) on
    every row; d_enc within 5e-2 on >= 99.9 % of rows (a ReLU input within rounding of 0
    can switch sides between two evaluation orders, changing that row's gradient path);
    parameter gradients (sums over 8.4 M rows) 2e-2 / 5e-2 relative L2."""
    from atmonr_amd import _lib

    width, nhd, nb, R, n_per_ray = 64, 2, 4, 8192, 1024
    M = R * n_per_ray
    bf = mma == "bf16"
    code = _lib.BF16 if bf else _lib.F16
    rtype = torch.bfloat16 if bf else torch.float16
    h = lambda t: t.to(rtype).float()
    rf, rg = (4e-2, 5e-2) if bf else (2e-2, 2e-2)
    g = torch.Generator(device=dev).manual_seed(11)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.nn.functional.normalize(torch.randn(R, 3, device=dev, generator=g), dim=1) * 0.5 + 0.5
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    sigma, color = torch.empty(M, device=dev), torch.empty(M, nb, device=dev)
    _lib.call("anr_ingp_field_fwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
              dirs.data_ptr(), n_per_ray, M, sigma.data_ptr(), color.data_ptr(), nb, s)
    dcol = torch.randn(M, nb, device=dev, generator=g) * 1e-3
    dsig = torch.randn(M, device=dev, generator=g) * 1e-3
    d_enc = torch.empty(M, 32, device=dev)
    g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, code, M)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    _lib.call("anr_ingp_field_bwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
              dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(), nb,
              d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), ws.data_ptr(),
              ws_bytes, s)
    # torch f32 reference with autograd
    e = enc.float().requires_grad_(True)
    tp, td = pp.clone().requires_grad_(True), pd.clone().requires_grad_(True)
    rs, rc = _field_torch_f32(e, dirs, n_per_ray, tp, td, width, nhd, nb, h)
    ((rc * dcol).sum() + (rs * dsig).sum()).backward()
    close(sigma, rs.detach(), rel=rf, atol=1e-5)
    close(color, rc.detach(), rel=rf, atol=1e-5)
    row_err = (d_enc - e.grad).abs().amax(1)
    ok = (row_err <= 5e-2 * e.grad.abs().max()).float().mean().item()
    assert ok >= 0.999, ok
    for a, b in ((g_pos, tp.grad), (g_dir, td.grad)):
        assert ((a - b).norm() / b.norm()).item() <= rg
    # 2,048 spot rows against the f64 CPU oracle (whole rays, so n_per_ray stays intact)
    rays = torch.randperm(R, generator=torch.Generator().manual_seed(3))[:2]
    rows = (rays[:, None] * n_per_ray + torch.arange(n_per_ray)[None]).reshape(-1).to(dev)
    half = "bf16" if bf else True
    rs64, rc64, _, _ = _field_ref(enc[rows].cpu().double(), dirs[rays.to(dev)].cpu().double(),
                                  n_per_ray, pp.cpu().double(), pd.cpu().double(), width, nhd,
                                  nb, half)
    close(sigma[rows], rs64, rel=rf, atol=1e-5)
    close(color[rows], rc64, rel=rf, atol=1e-5)


@pytest.mark.parametrize("tdt", ["f16", "f32"])
def test_hashgrid_fwd_v6_bit_identical_to_v1(dev, tdt):
    """The buffer-addressed walker (v6) and the walker (v1) evaluate the same corner order
    and fma chain: identical outputs, f16 and f32 tables, at a bench-like shape."""
    from atmonr_amd import _lib

    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    x = _grid_inputs(dev, (3, 16, 16, 1.3819, 19), 262144, True).to(dev)
    gen = torch.Generator(device=dev).manual_seed(5)
    dt = torch.float16 if tdt == "f16" else torch.float32
    table = ((torch.rand(d.n_params, device=dev, generator=gen) * 2 - 1) * 1e-2).to(dt)
    outs = []
    lib = _lib.load()
    for mode in (1, 0):  # v1, v6
        prev = lib.anr_hashgrid_force_v1(mode)
        out = torch.empty(x.shape[0], 32, device=dev, dtype=dt)
        _lib.call("anr_hashgrid_fwd", ctypes.byref(d), x.data_ptr(), 3, x.shape[0],
                  table.data_ptr(), _lib.dtype_code(dt), out.data_ptr(), _lib.dtype_code(dt),
                  32, _lib.stream(dev))
        lib.anr_hashgrid_force_v1(prev)
        outs.append(out)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)


@pytest.mark.parametrize("cfg,M,xs", [((3, 16, 16, 1.3819, 19), 100003, 3),
                                      ((3, 6, 4, 2.0, 10), 5001, 4),
                                      ((2, 16, 16, 1.3819, 19), 70001, 5),
                                      ((3, 16, 16, 1.3819, 19), 1, 3)])
@pytest.mark.parametrize("tdt", ["f16", "f32"])
def test_hashgrid_fwd_v6_outside_grid_and_strides(dev, cfg, M, xs, tdt):
    """v6 against v1, bit for bit, where v6's shortcuts matter: coordinates outside [0, 1]
    (dense levels wrap modulo T; the far-face test must send them down the exact path),
    coordinate and output row strides wider than the data, a ragged final chunk and a
    single sample (loads past the end of x return 0, stores past the last row drop)."""
    from atmonr_amd import _lib

    D, L = cfg[0], cfg[1]
    d = _lib.hashgrid_desc(D, L, 2, cfg[2], cfg[3], cfg[4])
    gen = torch.Generator(device=dev).manual_seed(11)
    R = -(-M // 97)
    o = torch.rand(R, 1, D, device=dev, generator=gen) * 2.0 - 0.5
    dr = (torch.rand(R, 1, D, device=dev, generator=gen) - 0.5) * 0.4
    t = torch.linspace(0, 1, 97, device=dev)[None, :, None]
    xx = (o + dr * t).reshape(-1, D)[:M]
    x = torch.zeros(M, xs, device=dev)
    x[:, :D] = xx
    x[::7, :D] = x[::7, :D].clamp(0, 1)  # exact faces too
    dt = torch.float16 if tdt == "f16" else torch.float32
    table = ((torch.rand(d.n_params, device=dev, generator=gen) * 2 - 1) * 1e-2).to(dt)
    lib = _lib.load()
    outs = []
    for mode in (1, 0):  # v1, v6 (default)
        prev = lib.anr_hashgrid_force_v1(mode)
        out = torch.full((M + 1, L * 2 + 3), -9.0, device=dev, dtype=dt)
        _lib.call("anr_hashgrid_fwd", ctypes.byref(d), x.data_ptr(), xs, M, table.data_ptr(),
                  _lib.dtype_code(dt), out.data_ptr(), _lib.dtype_code(dt), L * 2 + 3,
                  _lib.stream(dev))
        lib.anr_hashgrid_force_v1(prev)
        outs.append(out)
    for o_ in outs[1:]:
        assert torch.equal(outs[0], o_)
        assert torch.all(o_[:, L * 2:] == -9) and torch.all(o_[M] == -9)
    # the level-quad-plane entry point (v9, one lane per sample): the same values (f16
    # output) with level l, feature f of row m at out[(l // 4) * plane + 8 m + 2 (l % 4) + f],
    # a partial last quad zero-filled, nothing written past row M of a plane
    plane = 8 * M + 16
    nq = -(-L // 4)
    pl = torch.full((nq * plane + 8,), -9.0, device=dev, dtype=torch.float16)
    _lib.call("anr_hashgrid_fwd_planes", ctypes.byref(d), x.data_ptr(), xs, M,
              table.data_ptr(), _lib.dtype_code(dt), pl.data_ptr(), plane, _lib.stream(dev))
    got = torch.cat([pl[q * plane:q * plane + 8 * M].view(M, 8) for q in range(nq)], 1)
    assert torch.equal(got[:, :2 * L], outs[0][:M, :2 * L].half())
    assert torch.all(got[:, 2 * L:] == 0)
    for q in range(nq):
        assert torch.all(pl[q * plane + 8 * M:(q + 1) * plane] == -9)


@pytest.mark.parametrize("mma,ref", [("f16", False), ("bf16", False), ("f16", True)])
@pytest.mark.parametrize("n_per_ray,R,extra", [(1024, 5, 0), (64, 9, 13)])
def test_ingp_field_enc_quad_planes_equal_rows(dev, mma, ref, n_per_ray, R, extra):
    """The fused field reads its f16 hash features either in the row layout (M, 32) or in
    the level-quad planes anr_hashgrid_fwd_planes writes (enc_stride = -plane): forward,
    density, backward and the reference-numerics backward give bit-identical sigma /
    colour / dL/denc, and parameter gradients equal up to the atomic flush order."""
    from atmonr_amd import _lib

    width, nhd, nb = 64, 2, 4
    M = R * n_per_ray + extra
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    g = torch.Generator(device=dev).manual_seed(21)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    plane = 8 * M + 24
    planes = torch.zeros(4 * plane, device=dev, dtype=torch.float16)
    for q in range(4):
        planes[q * plane:q * plane + 8 * M] = enc[:, 8 * q:8 * q + 8].reshape(-1)
    dirs = torch.rand(R + 1, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dcol = (torch.randn(M, nb, device=dev, generator=g) * 1e-2).half().float()
    dsig = (torch.randn(M, device=dev, generator=g) * 1e-3).half().float()
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, code, M)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    out = {}
    for name, base, ld in (("rows", enc, 32), ("planes", planes, -plane)):
        sigma, color = torch.empty(M, device=dev), torch.empty(M, nb, device=dev)
        _lib.call("anr_ingp_field_fwd", pb, db, code, packed.data_ptr(), base.data_ptr(), ld,
                  dirs.data_ptr(), n_per_ray, M, sigma.data_ptr(), color.data_ptr(), nb, s)
        dens = torch.empty(M, device=dev)
        _lib.call("anr_ingp_field_density", pb, db, code, packed.data_ptr(), base.data_ptr(), ld,
                  M, dens.data_ptr(), s)
        d_enc = torch.empty(M, 32, device=dev)
        g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
        if ref:
            _lib.call("anr_ingp_field_bwd_ref16", pb, db, packed.data_ptr(), base.data_ptr(), ld,
                      dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), 128.0, s)
        else:
            _lib.call("anr_ingp_field_bwd", pb, db, code, packed.data_ptr(), base.data_ptr(), ld,
                      dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(),
                      ws.data_ptr() if ws_bytes else None, ws_bytes, s)
        out[name] = (sigma, color, dens, d_enc, g_pos, g_dir)
    for a, b in zip(out["rows"][:4], out["planes"][:4]):
        assert torch.equal(a, b)
    for a, b in zip(out["rows"][4:], out["planes"][4:]):
        assert (a - b).abs().max().item() <= 2e-5 * b.abs().max().item()
    with pytest.raises(_lib.ANRError):  # a plane shorter than 8 M rows is refused
        _lib.call("anr_ingp_field_fwd", pb, db, code, packed.data_ptr(), planes.data_ptr(),
                  -(8 * M - 8), dirs.data_ptr(), n_per_ray, M, sigma.data_ptr(),
                  color.data_ptr(), nb, s)


@pytest.mark.parametrize("ref", [False, True])
def test_ingp_field_bwd_zero_gradient_tiles(dev, ref):
    """Tiles whose incoming gradients are zero in every row are skipped by the field
    backward (r05). Rays with all-zero dL/dcolor and dL/dsigma (two 32-row tiles each,
    n_per_ray = 64) come back with dL/denc exactly 0, and the other rays' dL/denc equal a
    launch over those rays alone bit for bit (parameter gradients up to the atomic flush
    order; build numerics: within their per-wavefront gradient scale): skipping adds or
    drops nothing. Also a half-zero tile (walked). Build numerics (f16) and reference
    numerics (anr_ingp_field_bwd_ref16)."""
    from atmonr_amd import _lib

    width, nhd, nb, n_per_ray, R = 64, 2, 4, 64, 40
    M = R * n_per_ray
    g = torch.Generator(device=dev).manual_seed(8)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.rand(R, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, _lib.F16, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dcol = (torch.randn(M, nb, device=dev, generator=g) * 1e-2).half().float()
    dsig = (torch.randn(M, device=dev, generator=g) * 1e-3).half().float()
    zero_rays = [1, 2, 5, 11, 12, 13, 30, 39]
    zero = torch.zeros(M, dtype=torch.bool, device=dev)
    for r in zero_rays:
        zero[r * n_per_ray:(r + 1) * n_per_ray] = True
    dcol[zero], dsig[zero] = 0.0, 0.0
    dcol[20 * n_per_ray:20 * n_per_ray + 16] = 0.0   # half of a tile zero: walked
    dsig[20 * n_per_ray:20 * n_per_ray + 16] = 0.0

    def run(rays):
        rows = (torch.tensor(rays, device=dev)[:, None] * n_per_ray +
                torch.arange(n_per_ray, device=dev)[None]).reshape(-1)
        m = rows.numel()
        e_, dc, ds = enc[rows].contiguous(), dcol[rows].contiguous(), dsig[rows].contiguous()
        dr = dirs[torch.tensor(rays, device=dev)].contiguous()
        d_enc = torch.full((m, 32), float("nan"), device=dev)
        g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
        if ref:
            _lib.call("anr_ingp_field_bwd_ref16", pb, db, packed.data_ptr(), e_.data_ptr(), 32,
                      dr.data_ptr(), n_per_ray, m, ds.data_ptr(), dc.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), 128.0, s)
        else:
            ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, _lib.F16, m)
            ws = torch.empty(max(1, ws_bytes // 4), device=dev)
            _lib.call("anr_ingp_field_bwd", pb, db, _lib.F16, packed.data_ptr(), e_.data_ptr(),
                      32, dr.data_ptr(), n_per_ray, m, ds.data_ptr(), dc.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), ws.data_ptr(),
                      ws_bytes, s)
        return d_enc, g_pos, g_dir

    d_all, gp_all, gd_all = run(list(range(R)))
    live = [r for r in range(R) if r not in zero_rays]
    d_live, gp_live, gd_live = run(live)
    assert torch.all(d_all[zero] == 0)
    if ref:  # fixed gradient scale (128): every row's f16 chain is the same in both launches
        assert torch.equal(d_all[~zero], d_live.view(-1, 32))
        tol = 2e-5
    else:  # the build numerics' gradient scale is per wavefront, and the wavefronts differ
        assert (d_all[~zero] - d_live).abs().max().item() <= 1e-2 * d_live.abs().max().item()
        tol = 1e-2
    for a_, b_ in ((gp_all, gp_live), (gd_all, gd_live)):
        assert (a_ - b_).abs().max().item() <= tol * b_.abs().max().item()


@pytest.mark.parametrize("M", [262144, 1048576, 300000])
def test_hashgrid_bwd_tiles_equals_plain(dev, M):
    """anr_hashgrid_bwd_tiles skips the 32-row tiles flagged zero (the reference-numerics
    field backward's all-zero tiles) without loading them: with dL/dy zero on exactly those
    rows (plus tiles flagged 1 that are zero anyway, and a ragged end) the table gradient
    equals anr_hashgrid_bwd's up to the f32 atomic order. M = 300,000 has chunks that are
    not a multiple of 32 rows: the flags are ignored there (plain walker)."""
    from atmonr_amd import _lib

    cfg = (3, 16, 16, 1.3819, 19)
    d = _lib.hashgrid_desc(*cfg[:1], cfg[1], 2, cfg[2], cfg[3], cfg[4])
    x = _grid_inputs(dev, cfg, M, True).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    dout = torch.randn(M, 32, device=dev, generator=g) * 1e-3
    nt = -(-M // 32)
    flags = (torch.rand(nt, device=dev, generator=g) < 0.4).to(torch.uint8)
    rows_zero = flags.repeat_interleave(32)[:M] == 0
    dout[rows_zero] = 0.0
    flags[:: 7] = 1  # flagged walkable but zero where it was zeroed: still exact
    s = _lib.stream(dev)
    ga = torch.zeros(d.n_params, device=dev)
    gb = torch.zeros(d.n_params, device=dev)
    _lib.call("anr_hashgrid_bwd", ctypes.byref(d), x.data_ptr(), 3, M, dout.data_ptr(), _lib.F32,
              32, ga.data_ptr(), s)
    _lib.call("anr_hashgrid_bwd_tiles", ctypes.byref(d), x.data_ptr(), 3, M, dout.data_ptr(),
              _lib.F32, 32, gb.data_ptr(), flags.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.isfinite(gb).all()
    assert (ga - gb).abs().max().item() <= 1e-5 * ga.abs().max().item()
    assert ((ga != 0) == (gb != 0)).float().mean().item() > 0.9999


def _row_bits(d_enc):
    """Row bits as anr_ingp_field_bwd_ref16_rows writes them: bit m % 32 of word m // 32
    set iff row m has a nonzero value (int32 words)."""
    nz = (d_enc != 0).any(1).to(torch.int64).cpu()
    M = nz.numel()
    nz = torch.nn.functional.pad(nz, (0, -M % 32)).view(-1, 32)
    w = (nz << torch.arange(32, dtype=torch.int64)[None]).sum(1)
    return torch.where(w >= 2**31, w - 2**32, w).to(torch.int32)


@pytest.mark.parametrize("ws", [False, True])
@pytest.mark.parametrize("nb,n_per_ray,R", [(4, 64, 40), (4, 40, 13), (3, 64, 9), (4, 1024, 24)])
def test_ingp_field_bwd_ref16_rows_equals_f32_rows(dev, nb, n_per_ray, R, ws):
    """anr_ingp_field_bwd_ref16_rows (r06, ABI 5) against anr_ingp_field_bwd_ref16 on the
    same inputs: its f16 dL/denc rows hold exactly the f32 path's values (they are f16
    numbers: f16(f16(g_scaled) / 128)), bit for bit; its row bits are exactly the rows with
    a nonzero value; the parameter gradients agree up to the f32 atomic flush order. The
    inputs mix rays whose incoming gradients are zero (skipped tiles), rows whose tiny
    gradients underflow to zero dL/denc in f16, and ordinary rows; a ragged last tile
    (M = 520) and the general (non-fast) d_color layout (3 outputs) are covered. ws: with
    a workspace (the pos pass + list pass; every tile here has colour gradients, so the
    pos pass lists them all) and without (one kernel)."""
    from atmonr_amd import _lib

    width, nhd = 64, 2
    M = R * n_per_ray
    g = torch.Generator(device=dev).manual_seed(11)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.rand(R, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, _lib.F16, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dcol = (torch.randn(M, nb, device=dev, generator=g) * 1e-2).half().float()
    dsig = (torch.randn(M, device=dev, generator=g) * 1e-3).half().float()
    tiny = torch.rand(M, device=dev, generator=g) < 0.5
    dcol[tiny] *= 1e-5
    dsig[tiny] *= 1e-5
    for r in range(0, R, 3):
        dcol[r * n_per_ray:(r + 1) * n_per_ray] = 0.0
        dsig[r * n_per_ray:(r + 1) * n_per_ray] = 0.0
    outs = []
    for rows in (False, True):
        g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
        if rows:
            d_enc = torch.full((M, 32), float("nan"), device=dev, dtype=torch.float16)
            bits = torch.full((-(-M // 32),), -7, device=dev, dtype=torch.int32)
            wsb = lib.anr_ingp_field_bwd_ref16_rows_workspace_bytes(M) if ws else 0
            wst = torch.empty(max(1, wsb), device=dev, dtype=torch.uint8)
            _lib.call("anr_ingp_field_bwd_ref16_rows", pb, db, packed.data_ptr(), enc.data_ptr(),
                      32, dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), 128.0,
                      bits.data_ptr(), wst.data_ptr() if ws else None, wsb, s)
        else:
            d_enc = torch.full((M, 32), float("nan"), device=dev)
            bits = None
            _lib.call("anr_ingp_field_bwd_ref16", pb, db, packed.data_ptr(), enc.data_ptr(), 32,
                      dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), 128.0, s)
        outs.append((d_enc, bits, g_pos, g_dir))
    torch.cuda.synchronize()
    (d32, _, gp32, gd32), (d16, bits, gp16, gd16) = outs
    assert torch.equal(d16.float(), d32)
    nzr = (d32 != 0).any(1).float().mean().item()
    assert 0.05 < nzr < 0.95, nzr  # the mix above: both kinds of rows present
    assert torch.equal(bits.cpu(), _row_bits(d32))
    for a_, b_ in ((gp16, gp32), (gd16, gd32)):
        assert (a_ - b_).abs().max().item() <= 2e-5 * b_.abs().max().item()


@pytest.mark.parametrize("rows", [False, True, "ws"])
@pytest.mark.parametrize("n_per_ray,R", [(64, 40), (1024, 12), (1024, 300)])
def test_ingp_field_bwd_ref16_zero_color_tiles_skip_dir_net(dev, rows, n_per_ray, R):
    """Reference numerics (r06): a 32-row tile whose dL/dcolor is zero in every row skips
    the dir network's backward and the dir half of the forward recompute. Against the same
    launch with those zeros replaced by 1e-30 (nonzero, so the tile walks the dir network,
    whose f16 chain rounds them to exactly 0): dL/denc and the row bits are bit-identical and
    the parameter gradients agree up to the atomic flush order. Rays with ordinary colour
    gradients and rays with none (dL/dsigma too) are mixed in. rows = "ws": the f16-row
    kernel with a workspace, i.e. the pos pass (zero-colour tiles) + the list pass (the
    others), against the same launch on the 1e-30 inputs, where the pos pass lists every
    tile."""
    from atmonr_amd import _lib

    width, nhd, nb = 64, 2, 4
    M = R * n_per_ray
    g = torch.Generator(device=dev).manual_seed(12)
    lib = _lib.load()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.rand(R, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, _lib.F16, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dsig = (torch.randn(M, device=dev, generator=g) * 1e-3).half().float()
    dcol = torch.zeros(M, nb, device=dev)
    for r in range(0, R, 4):  # ordinary colour gradients on every 4th ray
        dcol[r * n_per_ray:(r + 1) * n_per_ray] = torch.randn(n_per_ray, nb, device=dev,
                                                              generator=g) * 1e-2
    dsig[n_per_ray:2 * n_per_ray] = 0.0  # ray 1: no gradient at all
    tiny = torch.where(dcol == 0, torch.full_like(dcol, 1e-30), dcol)
    outs = []
    for dc in (dcol, tiny):
        g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
        bits = None
        if rows:
            d_enc = torch.full((M, 32), float("nan"), device=dev, dtype=torch.float16)
            bits = torch.zeros(-(-M // 32), device=dev, dtype=torch.int32)
            wsb = lib.anr_ingp_field_bwd_ref16_rows_workspace_bytes(M) if rows == "ws" else 0
            wst = torch.empty(max(1, wsb), device=dev, dtype=torch.uint8)
            _lib.call("anr_ingp_field_bwd_ref16_rows", pb, db, packed.data_ptr(), enc.data_ptr(),
                      32, dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dc.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), 128.0,
                      bits.data_ptr(), wst.data_ptr() if wsb else None, wsb, s)
        else:
            d_enc = torch.full((M, 32), float("nan"), device=dev)
            _lib.call("anr_ingp_field_bwd_ref16", pb, db, packed.data_ptr(), enc.data_ptr(), 32,
                      dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dc.data_ptr(), nb,
                      d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(), 128.0, s)
        outs.append((d_enc, bits, g_pos, g_dir))
    torch.cuda.synchronize()
    (da, ba, gpa, gda), (db_, bb, gpb, gdb) = outs
    assert not torch.isnan(da).any()
    assert torch.equal(da, db_)
    assert (da != 0).any()
    if rows:
        assert torch.equal(ba, bb)
    assert (gpa - gpb).abs().max().item() <= 1e-5 * gpb.abs().max().item()
    assert (gda - gdb).abs().max().item() <= 1e-5 * gdb.abs().max().item()
    assert gdb.abs().max().item() > 0  # the rays with colour gradients reached the dir net


@pytest.mark.parametrize("M", [262144, 1048576, 300000, 8192 * 1024])
def test_hashgrid_bwd_rows_equals_plain(dev, M):
    """anr_hashgrid_bwd_rows (r06, ABI 5) walks only the rows whose bit is set: with f16
    dL/dy zero on ~70 % of the rows (in runs, as the settled reference numerics leave them)
    and the bits of exactly the nonzero rows, the table gradient equals anr_hashgrid_bwd's
    up to the f32 atomic order, with the clear rows filled with garbage (never read).
    Clearing the bits of some nonzero rows drops exactly those rows (== the plain walker on
    dL/dy with them zeroed). M = 300,000: chunks of 64 rows (the rule's 73 rounded down to
    whole 32-row words)."""
    from atmonr_amd import _lib

    cfg = (3, 16, 16, 1.3819, 19)
    d = _lib.hashgrid_desc(*cfg[:1], cfg[1], 2, cfg[2], cfg[3], cfg[4])
    x = _grid_inputs(dev, cfg, M, True).to(dev)
    g = torch.Generator(device=dev).manual_seed(4)
    dout = (torch.randn(M, 32, device=dev, generator=g) * 1e-3).half()
    runs = torch.rand(-(-M // 8), device=dev, generator=g) < 0.5
    zero = (runs.repeat_interleave(8)[:M]) | (torch.rand(M, device=dev, generator=g) < 0.4)
    dout[zero] = 0.0
    s = _lib.stream(dev)

    def walk(name, dy, bits=None):
        gt = torch.zeros(d.n_params, device=dev)
        args = [ctypes.byref(d), x.data_ptr(), 3, M, dy.data_ptr(), _lib.F16, 32, gt.data_ptr()]
        if bits is not None:
            args.append(bits.to(dev).data_ptr())
        _lib.call(name, *args, s)
        torch.cuda.synchronize()
        return gt

    ga = walk("anr_hashgrid_bwd", dout)
    # a clear row is never read: fill the clear rows with garbage for the row walker
    # (outside the walker's shapes they are zeroed in place first)
    dg = dout.clone()
    dg[zero] = 7.0
    gb = walk("anr_hashgrid_bwd_rows", dg, _row_bits(dout))
    assert torch.isfinite(gb).all()
    assert (ga - gb).abs().max().item() <= 1e-5 * ga.abs().max().item()
    assert ((ga != 0) == (gb != 0)).float().mean().item() > 0.9999
    drop = (~zero) & (torch.rand(M, device=dev, generator=g) < 0.2)
    dz = dout.clone()
    dz[drop] = 0.0
    gc = walk("anr_hashgrid_bwd_rows", dout.clone(), _row_bits(dz))
    gd = walk("anr_hashgrid_bwd", dz)
    assert (gc - gd).abs().max().item() <= 1e-5 * gd.abs().max().item()
    assert (gc - ga).abs().max().item() > 1e-3 * ga.abs().max().item()


def test_hashgrid_bwd_rows_outside_walker_zeroes_clear_rows(dev):
    """anr_hashgrid_bwd_rows on a shape outside its walker (here: the v1 kernels forced
    by the test hook) zeroes the clear rows of dL/dy in place, then walks every row: the
    same gradient as the plain walker on zeroed rows."""
    from atmonr_amd import _lib

    lib = _lib.load()
    M = 20000
    cfg = (3, 16, 16, 1.3819, 19)
    d = _lib.hashgrid_desc(*cfg[:1], cfg[1], 2, cfg[2], cfg[3], cfg[4])
    x = _grid_inputs(dev, cfg, M, True).to(dev)
    g = torch.Generator(device=dev).manual_seed(6)
    dout = (torch.randn(M, 32, device=dev, generator=g) * 1e-3).half()
    zero = torch.rand(M, device=dev, generator=g) < 0.6
    dout[zero] = 0.0
    dg = dout.clone()
    dg[zero] = 7.0
    s = _lib.stream(dev)
    ga, gb = torch.zeros(d.n_params, device=dev), torch.zeros(d.n_params, device=dev)
    prev = lib.anr_hashgrid_force_v1(1)
    try:
        _lib.call("anr_hashgrid_bwd", ctypes.byref(d), x.data_ptr(), 3, M, dout.data_ptr(),
                  _lib.F16, 32, ga.data_ptr(), s)
        _lib.call("anr_hashgrid_bwd_rows", ctypes.byref(d), x.data_ptr(), 3, M, dg.data_ptr(),
                  _lib.F16, 32, gb.data_ptr(), _row_bits(dout).to(dev).data_ptr(), s)
        torch.cuda.synchronize()
    finally:
        lib.anr_hashgrid_force_v1(prev)
    assert torch.equal(dg, dout)
    assert (ga - gb).abs().max().item() <= 1e-5 * ga.abs().max().item()


@pytest.mark.parametrize("mma", ["f16", "bf16"])
@pytest.mark.parametrize("width,nhd", [(64, 2), (64, 1), (32, 2)])
@pytest.mark.parametrize("R,n_per_ray", [(37, 64), (5, 1024), (8192, 1024)])
def test_hash_field_fwd_equals_two_kernels(dev, mma, width, nhd, R, n_per_ray):
    """anr_ingp_hash_field_fwd (r06: hash grid + field forward in one kernel) against
    anr_hashgrid_fwd_planes followed by anr_ingp_field_fwd on the planes: the planes it
    writes and sigma / colour are bit-identical, on ray-like coordinates (16 levels, T =
    2^19, f16 table), for every supported field shape, f16 and bf16 MFMA, a ragged ray count
    and the bench size (8,192 rays x 1,024 samples). Shapes outside its set (samples per ray
    not a multiple of 64) are refused with ANR_E_UNSUPPORTED."""
    from atmonr_amd import _lib

    if R == 8192 and (width, nhd, mma) != (64, 2, "f16"):
        pytest.skip("bench size: the bench's field only")
    M, nb = R * n_per_ray, 4
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    g = torch.Generator(device=dev).manual_seed(23)
    lib = _lib.load()
    d = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    o = torch.rand(R, 1, 3, device=dev, generator=g)
    dr = (torch.rand(R, 1, 3, device=dev, generator=g) - 0.5) * 0.6
    t = torch.linspace(0, 1, n_per_ray, device=dev)[None, :, None]
    x = (o + dr * t).clamp(0, 1).reshape(M, 3).contiguous()
    table = ((torch.rand(d.n_params, device=dev, generator=g) * 2 - 1) * 0.5).half()
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    dirs = torch.rand(R, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    out = {}
    for name in ("two", "fused"):
        planes = torch.full((4, M, 8), float("nan"), device=dev, dtype=torch.float16)
        sigma = torch.full((M,), float("nan"), device=dev)
        color = torch.full((M, nb), float("nan"), device=dev)
        if name == "two":
            _lib.call("anr_hashgrid_fwd_planes", ctypes.byref(d), x.data_ptr(), 3, M,
                      table.data_ptr(), _lib.F16, planes.data_ptr(), 8 * M, s)
            _lib.call("anr_ingp_field_fwd", pb, db, code, packed.data_ptr(), planes.data_ptr(),
                      -8 * M, dirs.data_ptr(), n_per_ray, M, sigma.data_ptr(),
                      color.data_ptr(), nb, s)
        else:
            _lib.call("anr_ingp_hash_field_fwd", ctypes.byref(d), x.data_ptr(), M,
                      table.data_ptr(), _lib.F16, planes.data_ptr(), 8 * M, pb, db, code,
                      packed.data_ptr(), dirs.data_ptr(), n_per_ray, sigma.data_ptr(),
                      color.data_ptr(), nb, s)
        torch.cuda.synchronize()
        out[name] = (planes, sigma, color)
    for a, b in zip(out["two"], out["fused"]):
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.float16 else a.view(torch.int32),
                           b.view(torch.int16) if b.dtype == torch.float16 else b.view(torch.int32))
    assert torch.isfinite(out["fused"][2]).all()
    rc = lib.anr_ingp_hash_field_fwd(ctypes.byref(d), x.data_ptr(), M, table.data_ptr(),
                                     _lib.F16, planes.data_ptr(), 8 * M, pb, db, code,
                                     packed.data_ptr(), dirs.data_ptr(), 48, sigma.data_ptr(),
                                     color.data_ptr(), nb, s)
    assert rc == -3  # ANR_E_UNSUPPORTED: 48 samples per ray
