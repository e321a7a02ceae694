"""The composite backward's per-32-row maxima of |dL/dcolor|, |dL/dsigma|
(anr_composite_bwd_tm) as the fused field backward's f16 gradient-scale input
(anr_ingp_field_bwd_tm), in place of the field's own max-reduction pass over the same
gradients (absmax_kernel). max is exact, so the scale and every result must be the ones
of the two-pass form: bit-identical dL/denc, parameter gradients up to the f32 atomic
flush order. Composite: graphics_utils.py:6-77 (render_with_surface's backward)."""

import ctypes

import pytest
import torch

import __graft_entry__ as ge

pytestmark = pytest.mark.gpu


def _composite_inputs(dev, B, N, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    z = torch.sort(torch.rand(B, N, device=dev, generator=g) * 20.0, dim=1).values
    color = torch.rand(B, N, 4, device=dev, generator=g)
    sigma = torch.rand(B, N, 1, device=dev, generator=g) * 0.3
    cs = torch.rand(B, 4, device=dev, generator=g)
    g_cm = torch.randn(B, 4, device=dev, generator=g)
    return z, color, sigma, cs, g_cm


@pytest.mark.parametrize("N", [32, 64, 96, 224, 256, 288, 512, 1024, 2048])
def test_composite_tile_max_is_max_of_its_gradients(dev, N):
    from atmonr_amd import _lib

    lib = _lib.load()
    assert lib.anr_composite_tile_max_supported(_lib.F32, N, 4, 1) == 1
    B = 5
    z, color, sigma, cs, g_cm = _composite_inputs(dev, B, N, N)
    s = _lib.stream(dev)
    outs = []
    for tm_on in (False, True):
        d_color = torch.full_like(color, float("nan"))
        d_sigma = torch.full_like(sigma, float("nan"))
        d_z = torch.empty(B, N, device=dev)
        args = [z.data_ptr(), 0.5, color.data_ptr(), sigma.data_ptr(), cs.data_ptr(), _lib.F32,
                B, N, 4, 1, g_cm.data_ptr(), None, None, None, None, d_color.data_ptr(),
                d_sigma.data_ptr(), None, d_z.data_ptr()]
        if tm_on:
            tm = torch.full((B * N // 32,), -1.0, device=dev)
            _lib.call("anr_composite_bwd_tm", *args, tm.data_ptr(), s)
        else:
            tm = None
            _lib.call("anr_composite_bwd", *args, s)
        outs.append((d_color, d_sigma, d_z, tm))
    (c0, s0, z0, _), (c1, s1, z1, tm) = outs
    assert torch.equal(c0, c1) and torch.equal(s0, s1) and torch.equal(z0, z1)
    want = torch.maximum(c1.abs().amax(-1), s1.abs()[..., 0]).reshape(-1, 32).amax(-1)
    assert torch.equal(tm, want)


@pytest.mark.parametrize("N", [16, 100, 160, 4100])
def test_composite_tile_max_unsupported_shapes(dev, N):
    """Rays that are not whole 32-row tiles, lanes whose samples straddle a tile (SPL = 3)
    and rays past the register-blocked kernels: not offered, and the entry point refuses."""
    from atmonr_amd import _lib

    lib = _lib.load()
    assert lib.anr_composite_tile_max_supported(_lib.F32, N, 4, 1) == 0
    assert lib.anr_composite_tile_max_supported(_lib.F16, 1024, 4, 1) == 0
    assert lib.anr_composite_tile_max_supported(_lib.F32, 1024, 4, 4) == 0
    z, color, sigma, cs, g_cm = _composite_inputs(dev, 2, N, 1)
    d_color, d_sigma = torch.empty_like(color), torch.empty_like(sigma)
    tm = torch.empty(max(1, 2 * N // 32), device=dev)
    with pytest.raises(_lib.ANRError):
        _lib.call("anr_composite_bwd_tm", z.data_ptr(), 0.5, color.data_ptr(), sigma.data_ptr(),
                  cs.data_ptr(), _lib.F32, 2, N, 4, 1, g_cm.data_ptr(), None, None, None, None,
                  d_color.data_ptr(), d_sigma.data_ptr(), None, None, tm.data_ptr(),
                  _lib.stream(dev))


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("extra", [0, 29])
def test_field_bwd_tile_max_equals_two_pass(dev, mode, extra):
    from atmonr_amd import _lib

    nb, R, n_per_ray, width, nhd = 4, 64, 256, 64, 2
    M = R * n_per_ray + extra
    code = _lib.F16
    g = torch.Generator(device=dev).manual_seed(7 + extra)
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
    # gradients spanning decades, so tiles (and waves) get different scales
    dcol = torch.randn(M, nb, device=dev, generator=g) * 10.0 ** torch.randint(
        -6, 0, (M, 1), device=dev, generator=g).float()
    dsig = torch.randn(M, device=dev, generator=g) * 1e-3
    pad = (-M) % 32
    rowmax = torch.maximum(dcol.abs().amax(1), dsig.abs())
    tm = torch.cat([rowmax, rowmax.new_zeros(pad)]).view(-1, 32).amax(1).contiguous()
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, code, M)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    prev = lib.anr_ingp_field_force_bwd(mode)
    try:
        res = []
        for use_tm in (False, True):
            d_enc = torch.empty(M, 32, device=dev)
            g_pos, g_dir = torch.zeros_like(pp), torch.zeros_like(pd)
            if use_tm:
                _lib.call("anr_ingp_field_bwd_tm", pb, db, code, packed.data_ptr(),
                          enc.data_ptr(), 32, dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(),
                          dcol.data_ptr(), nb, tm.data_ptr(), d_enc.data_ptr(), 32,
                          g_pos.data_ptr(), g_dir.data_ptr(), s)
            else:
                _lib.call("anr_ingp_field_bwd", pb, db, code, packed.data_ptr(), enc.data_ptr(),
                          32, dirs.data_ptr(), n_per_ray, M, dsig.data_ptr(), dcol.data_ptr(),
                          nb, d_enc.data_ptr(), 32, g_pos.data_ptr(), g_dir.data_ptr(),
                          ws.data_ptr(), ws_bytes, s)
            res.append((d_enc, g_pos, g_dir))
    finally:
        lib.anr_ingp_field_force_bwd(prev)
    (e0, p0, q0), (e1, p1, q1) = res
    assert torch.equal(e0, e1)
    for a, b in ((p1, p0), (q1, q0)):
        assert (a - b).abs().max().item() <= 2e-5 * b.abs().max().item()


def test_pipeline_step_hands_tile_max_to_field(dev, monkeypatch):
    """With the hand-off on (ANR_TILE_MAX=1) the composite's maxima reach the fused field
    backward in the Instant-NGP train step (the field runs no max pass of its own), and the
    gradients equal the two-pass step."""
    from atmonr_amd import field as field_mod
    from atmonr_amd import graphics_utils
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    scene = SyntheticHARP2Dataset(n_views=4, img_size=32, device=dev, seed=0)
    batch = next(iter(BatchLoader(scene, 256, seed=1)))
    u = torch.rand(256, 128, device=dev)
    grads, taken = [], []
    monkeypatch.setattr(graphics_utils, "_TILE_MAX_ON", True)
    real = field_mod.take_tile_max
    for hand_off in (True, False):
        def spy(dc, ds, _on=hand_off):
            tm = real(dc, ds)
            taken.append(tm is not None)
            return tm if _on else None

        monkeypatch.setattr(field_mod, "take_tile_max", spy)
        p = InstantNGPPipeline(ge._ingp_config(128), scene, dtype=torch.float16, fused=True,
                               seed=5)
        p.send_tensors_to(dev)
        res = p.forward(batch, u=u)
        p.compute_loss(batch, res).backward()
        grads.append([q.grad.detach().clone() for q in p.parameters() if q.grad is not None])
    assert taken == [True, True]  # offered on both runs; used on the first only
    assert len(grads[0]) == len(grads[1]) > 0
    for a, b in zip(*grads):
        assert (a - b).abs().max().item() <= 2e-5 * max(b.abs().max().item(), 1e-30)
