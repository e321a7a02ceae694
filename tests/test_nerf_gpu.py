"""NeRF path on the GPU against the reference's golden vectors and the
oracle (oracle/ref_nerf.py, oracle/ref_path.py) on identical inputs and random draws."""

import numpy as np
import pytest
import torch

from tests.conftest import golden
from oracle import ref_nerf, ref_path

pytestmark = pytest.mark.gpu


def close(a, b, rel, atol, what=""):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item() if a.numel() else 0.0
    tol = rel * b.abs().max().item() + atol
    assert err <= tol, f"{what}: max err {err:.3e} > tol {tol:.3e}"


def test_posenc_matches_reference_golden(dev):
    from atmonr_amd.encoders import positional_encoding

    g = golden("nerf.npz")
    pts = torch.from_numpy(g["pe_pts"]).to(dev)
    out = positional_encoding(pts, [14, 14, 10])
    assert out.shape == (3, 11, 76)
    close(out, g["pe_list"], rel=0, atol=2e-5)
    dirs = torch.from_numpy(g["pe_dirs"]).to(dev)
    out = positional_encoding(dirs, 4)
    assert out.shape == (33, 3, 8)
    close(out, g["pe_int"], rel=0, atol=2e-6)


@pytest.mark.parametrize("L", [[14, 14, 10], 4])
def test_posenc_grad_matches_oracle(dev, L):
    from atmonr_amd.encoders import positional_encoding

    gen = torch.Generator().manual_seed(3)
    x = torch.rand(500, 3, generator=gen) * 2 - 1
    xr = x.clone().requires_grad_(True)
    ref = ref_path.positional_encoding(xr, L)
    dout = torch.randn(ref.shape, generator=gen)
    (ref * dout).sum().backward()
    xd = x.to(dev).requires_grad_(True)
    out = positional_encoding(xd, L)
    close(out, ref.detach(), rel=0, atol=2e-5)
    (out * dout.to(dev)).sum().backward()
    close(xd.grad, xr.grad, rel=2e-5, atol=1e-3)


def test_sample_pdf_matches_reference_golden(dev):
    from atmonr_amd.samplers import sample_pdf

    g = golden("sample_pdf.npz")
    t = {k: torch.from_numpy(g[k]).to(dev) for k in g.files}
    pts, z = sample_pdf({"origin": t["origin"], "dir": t["dir"]}, t["w"], t["zc"], 128, u=t["u"])
    assert torch.equal(z.cpu(), torch.from_numpy(g["z"]))
    assert torch.equal(pts.cpu(), torch.from_numpy(g["pts"]))


def test_sample_pdf_grad_matches_oracle(dev):
    from atmonr_amd.samplers import sample_pdf

    gen = torch.Generator().manual_seed(11)
    B, Nc, Nf = 37, 64, 128
    origin = torch.randn(B, 3, generator=gen)
    direction = torch.nn.functional.normalize(torch.randn(B, 3, generator=gen), dim=1)
    zc = torch.sort(torch.rand(B, Nc, generator=gen), dim=1).values * 3
    w = torch.rand(B, Nc, 1, generator=gen) ** 4
    w[:5, 10:30] = 0.0  # empty bins: denom < 1e-8 branch
    u = torch.rand(B, Nf, generator=gen)
    wr = w.clone().requires_grad_(True)
    pr, zr = ref_nerf.sample_pdf(origin, direction, wr, zc, Nf, u=u)
    gp, gz = torch.randn(pr.shape, generator=gen), torch.randn(zr.shape, generator=gen)
    ((pr * gp).sum() + (zr * gz).sum()).backward()
    wd = w.to(dev).requires_grad_(True)
    p, z = sample_pdf({"origin": origin.to(dev), "dir": direction.to(dev)}, wd, zc.to(dev), Nf,
                      u=u.to(dev))
    close(z, zr.detach(), rel=1e-6, atol=1e-7)
    close(p, pr.detach(), rel=1e-6, atol=1e-6)
    ((p * gp.to(dev)).sum() + (z * gz.to(dev)).sum()).backward()
    close(wd.grad, wr.grad, rel=1e-4, atol=1e-6)


def _prep_kwargs(pp):
    return dict(scale=float(pp.scale), offset=torch.tensor(pp.offset, dtype=torch.float64),
                lat_min=pp.lat_min, lat_range=pp.lat_range, lon_min=pp.lon_min,
                lon_range=pp.lon_range, h0=pp.ray_origin_height, shift_lon=pp.shift_lon)


@pytest.fixture(scope="module")
def scene(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    return SyntheticHARP2Dataset(n_views=8, img_size=32, device=dev, seed=0)


def test_preprocess_bwd_matches_torch_autograd(scene, dev):
    from atmonr_amd.samplers import preprocess_points

    pp = scene.get_point_preprocessor("horizontal")
    gen = torch.Generator().manual_seed(5)
    pts = (torch.rand(4000, 3, generator=gen) * 2 - 1) * torch.tensor([1.0, 1.0, 0.3])
    pts[:50] *= 1.5  # some points outside the scene box: clipped coordinates
    pr = pts.clone().requires_grad_(True)
    ref = ref_nerf.preprocess_torch(pr, **_prep_kwargs(pp))
    g = torch.randn(ref.shape, generator=gen)
    (ref * g).sum().backward()
    pd = pts.to(dev).requires_grad_(True)
    out = preprocess_points(pd, pp.params())
    close(out, ref.detach(), rel=0, atol=2e-6)
    (out * g.to(dev)).sum().backward()
    close(pd.grad, pr.grad, rel=1e-4, atol=1e-4)


NERF_CFG = {"type": "NeRF", "include_height": False, "point_preprocessor": "horizontal",
            "num_bands": 4, "ray_origin_height": 20000, "sampler": {"N_c": 64, "N_f": 128},
            "encoder": {"L_x": [14, 14, 10], "L_d": 4}, "mlp_hidden_dim": 64}


def _oracle_step(pipe_sd, pp, scale, batch, u_c, u_f, noise, train, w_coarse_dev,
                 dtype=torch.float32):
    """nerf.py train step op by op with the oracle functions, identical draws, computed in
    ``dtype``. The fine sampler sees the device's coarse-weight values (its inverse-cdf is
    steep in narrow bins, so GEMM-order differences upstream would move z by more than
    the sampler's own error) while the gradient still flows through the oracle's coarse
    weights."""
    L_x, L_d = NERF_CFG["encoder"]["L_x"], NERF_CFG["encoder"]["L_d"]
    nets = {}
    for mode, V in (("coarse", 1), ("fine", 4)):
        n = ref_nerf.RefAtmoNeRF(76, 24, 4, V, NERF_CFG["mlp_hidden_dim"])
        n.load_state_dict({k: v.cpu() for k, v in pipe_sd[mode].items()})
        n.to(dtype).train(train)
        nets[mode] = n
    b = {k: (v.cpu().to(dtype) if v.is_floating_point() else v.cpu()) for k, v in batch.items()}
    u_c, u_f = u_c.to(dtype), u_f.to(dtype)
    B = b["origin"].shape[0]
    res = {}
    w_c = z_c = None
    for mode in ("coarse", "fine"):
        if mode == "coarse":
            N = 64
            bins = torch.linspace(0, 1, N + 1, dtype=dtype)[None]
            z = (bins[:, :-1] + u_c / N) * b["len"][:, None]
            pts = b["origin"][:, None] + b["dir"][:, None] * z[..., None]
        else:
            N = 192
            w_in = w_c + (w_coarse_dev.detach().cpu().to(dtype) - w_c).detach()
            pts, z = ref_nerf.sample_pdf(b["origin"], b["dir"], w_in, z_c, 128, u=u_f)
        pts = ref_nerf.preprocess_torch(pts, **_prep_kwargs(pp))
        pe = ref_path.positional_encoding(pts, L_x).view(B * N, -1)
        de = ref_path.positional_encoding(b["dir"][:, None].repeat(1, N, 1), L_d).view(B * N, -1)
        net = nets[mode]
        x = torch.cat([pe, de], dim=1)
        # RefAtmoNeRF adds torch.randn in training mode; replay the injected noise instead
        xp, d = x[:, :76], x[:, 76:]
        h = xp
        for i in range(1, 6):
            h = torch.relu(getattr(net, f"fc{i}")(h))
        h = torch.cat([h, xp], dim=1)
        for i in range(6, 9):
            h = torch.relu(getattr(net, f"fc{i}")(h))
        h = net.fc9(h)
        sigma = h[:, net.hidden_dim:]
        if train:
            sigma = sigma + noise[mode].cpu().to(dtype)
        sigma = torch.relu(sigma)
        hh = torch.relu(net.fc10(torch.cat([h[:, : net.hidden_dim], d], dim=1)))
        color = torch.sigmoid(net.fc11(hh))
        color = torch.exp(torch.clamp(color.view(B, N, -1), max=11))
        sigma = torch.relu(sigma.view(B, N, -1))
        cm, _, w = ref_path.render(z * (scale / 1000), color, sigma)
        res[mode] = (cm, w, z)
        w_c, z_c = w, z
    idx = b["irgb_idx"][:, None]
    loss = sum(torch.nn.functional.mse_loss(torch.take_along_dim(res[m][0], idx, 1)[:, 0],
                                            b["rad"]) for m in ("coarse", "fine"))
    loss.backward()
    grads = {m: {k: p.grad for k, p in nets[m].named_parameters()} for m in nets}
    return res, loss.detach(), grads


@pytest.mark.parametrize("train", [False, True])
def test_nerf_pipeline_matches_oracle(scene, dev, train):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.pipelines.factory import get_pipeline

    torch.manual_seed(0)
    pipe = get_pipeline(NERF_CFG, scene)
    pipe.send_tensors_to(dev)
    pipe.train() if train else pipe.eval()
    batch = next(iter(BatchLoader(scene, 96, seed=2)))
    gen = torch.Generator().manual_seed(9)
    B = batch["origin"].shape[0]
    u_c, u_f = torch.rand(B, 64, generator=gen), torch.rand(B, 128, generator=gen)
    noise = {"coarse": torch.randn(B * 64, 1, generator=gen),
             "fine": torch.randn(B * 192, 4, generator=gen)}
    res = pipe.forward(batch, u_coarse=u_c.to(dev), u_fine=u_f.to(dev),
                       noise={k: v.to(dev) for k, v in noise.items()})
    loss = pipe.compute_loss(batch, res)
    loss.backward()
    ref, ref_loss, ref_grads = _oracle_step(pipe.state_dict(), scene.get_point_preprocessor(
        "horizontal"), pipe.scale, batch, u_c, u_f, noise, train, res["weights_coarse"])
    for mode in ("coarse", "fine"):
        cm, w, z = ref[mode]
        close(res[f"z_vals_{mode}"], z.detach(), rel=1e-6, atol=1e-6, what=f"z_{mode}")
        close(res[f"color_map_{mode}"], cm.detach(), rel=2e-4, atol=1e-6, what=f"cm_{mode}")
        close(res[f"weights_{mode}"], w.detach(), rel=2e-4, atol=1e-6, what=f"w_{mode}")
    close(loss.detach(), ref_loss, rel=2e-4, atol=0, what="loss")
    # Gradients: the coarse net's gradient passes through sample_pdf's t_in_bin, whose
    # 1/denom terms cancel in the cumsum backward; the f32 autograd of the reference is
    # itself noisy there in narrow bins. Judge both against an f64 oracle: the device
    # (fp64 accumulation in that backward) must be within the tolerance plus twice the
    # reference-precision error.
    _, _, g64 = _oracle_step(pipe.state_dict(), scene.get_point_preprocessor("horizontal"),
                             pipe.scale, batch, u_c, u_f, noise, train, res["weights_coarse"],
                             dtype=torch.float64)
    for mode in ("coarse", "fine"):
        for k, p in pipe.nerf[mode].named_parameters():
            exact = g64[mode][k]
            e_dev = (p.grad.double().cpu() - exact).abs().max().item()
            e_ref = (ref_grads[mode][k].double() - exact).abs().max().item()
            tol = 5e-3 * exact.abs().max().item() + 1e-7 + 2 * e_ref
            assert e_dev <= tol, f"d{mode}.{k}: err {e_dev:.3e} > {tol:.3e} (f32 ref {e_ref:.3e})"


def test_nerf_training_reduces_loss(scene, dev):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.pipelines.factory import get_pipeline

    torch.manual_seed(1)
    pipe = get_pipeline(NERF_CFG, scene)
    pipe.send_tensors_to(dev)
    opt = pipe.get_optimizer({"lr": 5e-4})
    loader = BatchLoader(scene, 512, seed=3)
    # NeRF colours are exp(sigmoid(.)) in (1, e) (nerf.py:150): rescale the synthetic
    # radiance into the range the model can express
    k = 2.5 / scene.max_i
    losses = []
    for _, batch in zip(range(60), iter(loader)):
        batch = dict(batch, rad=batch["rad"] * k)
        res = pipe.forward(batch)
        loss = pipe.compute_loss(batch, res)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert np.isfinite(losses).all()
    assert np.mean(losses[-10:]) < 0.8 * np.mean(losses[:10]), losses
    sig = pipe.extract(torch.rand(1000, 3, device=dev) * 2 - 1)
    assert sig.shape == (1000, 4) and bool((sig >= 0).all())


@pytest.mark.parametrize("M,C", [(786432, 256), (262144, 128), (5000, 12), (300, 1024), (0, 8)])
def test_relu_bwd_colsum_matches_torch(dev, M, C):
    """anr_relu_bwd_colsum (AtmoNeRF Linear+ReLU backward): the masked gradient equals
    torch's threshold_backward bit for bit; the bias gradient (sum of the per-block
    partials) equals g'.sum(0) in f64 within f32 summation error (1e-5 of sum |g'|)."""
    from atmonr_amd import _lib

    gen = torch.Generator(device=dev).manual_seed(M + C)
    g = torch.randn(M, C, device=dev, generator=gen)
    y = torch.relu(torch.randn(M, C, device=dev, generator=gen))
    parts = max(1, min(1024, M // 256))
    gm = torch.empty_like(g)
    partial = torch.full((parts, C), float("nan"), device=dev)
    _lib.call("anr_relu_bwd_colsum", _lib.ptr(g), _lib.ptr(y), M, C, _lib.ptr(gm),
              _lib.ptr(partial), parts, _lib.stream(dev))
    ref = torch.ops.aten.threshold_backward(g, y, 0)
    assert torch.equal(gm, ref)
    db = partial.sum(0).double()
    want = ref.double().sum(0)
    assert torch.all((db - want).abs() <= 1e-5 * ref.double().abs().sum(0) + 1e-30)


# ------------------------------------------------------------------ AtmoNeRF dense layers
# csrc/nerf_mlp.hip against f64 torch on the same f32 operands: f32 MFMA sums in another
# order than hipBLASLt's, so the bar is f32 summation error (rel 1e-5 of sum |a·b| terms).
def _f32_bar(a, b):
    return 2e-5 * (a.double().abs() @ b.double().abs().t()) + 1e-30


def _pack_bits(mask):
    """(M, C) bool -> (M, ceil(C/64)) int64 words in the kernels' layout: column
    64w + 16j + 4g + r is bit 16g + 4j + r of word w (csrc/nerf_mlp.hip)."""
    M, C = mask.shape
    W = (C + 63) // 64
    m = torch.zeros(M, W * 64, dtype=torch.int64, device=mask.device)
    m[:, :C] = mask.long()
    k = torch.arange(64, device=mask.device, dtype=torch.int64)
    j, g, r = k // 16, (k % 16) // 4, k % 4
    shifts = 16 * g + 4 * j + r
    return (m.view(M, W, 64) << shifts).sum(-1)


@pytest.mark.parametrize("M,q1,q2,n,relu", [(1000, 76, 0, 256, 1), (4096, 256, 76, 256, 1),
                                            (777, 256, 24, 128, 1), (300, 256, 0, 257, 0),
                                            (64, 128, 0, 4, 0), (70000, 256, 0, 256, 1),
                                            (0, 256, 0, 256, 1)])
def test_nerf_linear_fwd_matches_f64(dev, M, q1, q2, n, relu):
    """Y = [A1 | A2] W^T + b (+ ReLU), the pad columns zero, and the ReLU bitmask equal to
    (Y > 0) bit for bit."""
    from atmonr_amd import _lib

    gen = torch.Generator(device=dev).manual_seed(M + n)
    lda = q1 + q2 + 4       # strided rows, as the encoding and the padded fc9 output are
    x = torch.randn(M, lda, device=dev, generator=gen)
    w = torch.randn(n, q1 + q2, device=dev, generator=gen) * 0.1
    b = torch.randn(n, device=dev, generator=gen)
    ld = (n + 3) // 4 * 4
    y = torch.full((M, ld), float("nan"), device=dev)
    bits = torch.full((M, (n + 63) // 64), -1, dtype=torch.int64, device=dev) if relu else None
    a2 = x[:, q1:] if q2 else None
    _lib.call("anr_nerf_linear_fwd", _lib.ptr(x), lda, q1, _lib.ptr(a2), lda, q2, M,
              _lib.ptr(w), n, _lib.ptr(b), relu, _lib.ptr(y), ld, _lib.ptr(bits),
              _lib.stream(dev))
    a = x[:, : q1 + q2]
    want = a.double() @ w.double().t() + b.double()
    bar = _f32_bar(a, w) + 1e-6 * b.double().abs()
    if relu:
        want = want.clamp_min(0)
    assert torch.all((y[:, :n].double() - want).abs() <= bar)
    assert torch.all(y[:, n:] == 0)
    if relu:
        assert torch.equal(bits, _pack_bits(y[:, :n] > 0))


@pytest.mark.parametrize("M,n,p1,p2,acc2", [(1000, 256, 256, 76, 0), (1000, 256, 0, 76, 1),
                                            (555, 257, 256, 0, 0), (300, 4, 128, 0, 0),
                                            (4096, 128, 0, 256, 0), (70001, 256, 256, 0, 0)])
def test_nerf_linear_dx_matches_f64(dev, M, n, p1, p2, acc2):
    """dX = G W with the ReLU bitmask applied to the first p1 columns (exactly zero where
    the bit is clear, as torch's threshold_backward) and an accumulating second segment."""
    from atmonr_amd import _lib

    gen = torch.Generator(device=dev).manual_seed(M + n + p1)
    nr = (n + 3) // 4 * 4
    g = torch.zeros(M, nr, device=dev)
    g[:, :n] = torch.randn(M, n, device=dev, generator=gen)
    w = torch.randn(n, p1 + p2, device=dev, generator=gen) * 0.1
    wt = torch.zeros(p1 + p2, nr, device=dev)
    wt[:, :n] = w.t()
    keep = torch.rand(M, max(p1, 1), device=dev, generator=gen) > 0.4
    bits = _pack_bits(keep[:, :p1]) if p1 else None
    dx1 = torch.full((M, max(p1, 1)), float("nan"), device=dev)
    base = torch.randn(M, p2 + 4, device=dev, generator=gen)
    dx2 = base.clone()
    _lib.call("anr_nerf_linear_dx", _lib.ptr(g), nr, M, n, _lib.ptr(wt), nr, p1, p2,
              _lib.ptr(bits), _lib.ptr(dx1) if p1 else None, dx1.stride(0),
              _lib.ptr(dx2) if p2 else None, dx2.stride(0), acc2, _lib.stream(dev))
    full = g[:, :n].double() @ w.double()
    bar = _f32_bar(g[:, :n], w.t())
    if p1:
        k = keep[:, :p1]
        want = torch.where(k, full[:, :p1], torch.zeros_like(full[:, :p1]))
        assert torch.all((dx1[:, :p1].double() - want).abs() <= bar[:, :p1])
        assert torch.all(dx1[:, :p1][~k] == 0)
    if p2:
        want2 = full[:, p1:] + (base[:, :p2].double() if acc2 else 0)
        assert torch.all((dx2[:, :p2].double() - want2).abs()
                         <= bar[:, p1:] + 1e-6 * base[:, :p2].double().abs())
        assert torch.equal(dx2[:, p2:], base[:, p2:])


@pytest.mark.parametrize("M,n,q1,q2", [(786432, 256, 256, 0), (1000, 257, 256, 0),
                                       (4099, 128, 256, 24), (5000, 256, 256, 76),
                                       (300, 4, 128, 0), (0, 256, 76, 0)])
def test_nerf_linear_dw_matches_f64(dev, M, n, q1, q2):
    """dW += G^T [A1 | A2] and db += colsum(G), accumulated, deterministic (two launches
    give identical bits)."""
    from atmonr_amd import _lib

    gen = torch.Generator(device=dev).manual_seed(M + n + q2)
    nr = (n + 3) // 4 * 4
    g = torch.zeros(M, nr, device=dev)
    g[:, :n] = torch.randn(M, n, device=dev, generator=gen)
    lda = q1 + q2 + 8
    x = torch.randn(M, lda, device=dev, generator=gen)
    K = q1 + q2
    dw0 = torch.randn(n, K, device=dev, generator=gen)
    db0 = torch.randn(n, device=dev, generator=gen)
    lib = _lib.load()
    ws = torch.empty(max(16, lib.anr_nerf_linear_dw_workspace(M, n, K)) // 4, device=dev)
    outs = []
    for _ in range(2):
        dw, db = dw0.clone(), db0.clone()
        _lib.call("anr_nerf_linear_dw", _lib.ptr(g), nr, M, n, _lib.ptr(x), lda, q1,
                  _lib.ptr(x[:, q1:]) if q2 else None, lda, q2, _lib.ptr(dw), _lib.ptr(db),
                  _lib.ptr(ws), ws.numel() * 4, _lib.stream(dev))
        outs.append((dw, db))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    dw, db = outs[0]
    gd, xd = g[:, :n].double(), x[:, :K].double()
    want = dw0.double() + gd.t() @ xd
    bar = 2e-5 * (gd.abs().t() @ xd.abs()) + 1e-6 * dw0.double().abs() + 1e-30
    assert torch.all((dw.double() - want).abs() <= bar)
    wantb = db0.double() + gd.sum(0)
    assert torch.all((db.double() - wantb).abs() <= 2e-5 * gd.abs().sum(0) + 1e-6 * db0.double().abs() + 1e-30)


@pytest.mark.parametrize("vol,M", [(1, 4096 * 2 + 7), (4, 3000)])
def test_atmonerf_native_matches_library_path(dev, vol, M):
    """AtmoNeRF.forward on csrc/nerf_mlp.hip (_AtmoNeRFFn) against the library-GEMM path
    (torch.nn.Linear, autograd) on the same parameters, inputs and noise: outputs and every
    gradient (parameters and dL/dx_pos, the fc1 + fc6 skip sum) within f32 GEMM
    rounding."""
    from atmonr_amd import nerf_model

    torch.manual_seed(7)
    net = nerf_model.AtmoNeRF(76, 24, 4, vol, 256).to(dev)
    net.train()
    gen = torch.Generator(device=dev).manual_seed(M)
    x0 = torch.randn(M, 100, device=dev, generator=gen)
    noise = torch.randn(M, vol, device=dev, generator=gen)
    dcol = torch.randn(M, 4, device=dev, generator=gen)
    dsig = torch.randn(M, vol, device=dev, generator=gen)
    res = {}
    for mode in ("native", "torch"):
        nerf_model._NATIVE = mode == "native"
        try:
            net.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            color, sigma = net(x, noise)
            ((color * dcol).sum() + (sigma * dsig).sum()).backward()
            res[mode] = (color.detach(), sigma.detach(), x.grad.clone(),
                         [p.grad.clone() for p in net.params_in_order()])
        finally:
            nerf_model._NATIVE = True
    (cn, sn, xn, gn), (ct, s_t, xt, gt) = res["native"], res["torch"]
    close(cn, ct, rel=1e-4, atol=1e-6, what="color")
    close(sn, s_t, rel=1e-4, atol=1e-5, what="sigma")

    def rel_l2(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    # gradients: relative L2. A pre-activation within f32 rounding of 0 can take the
    # ReLU's other branch in the two summation orders, which moves that row's backward
    # by O(|g w|): elementwise bars would test the branch, not the kernels (measured on
    # MI355X: one dL/dx element 3e-2 apart on a max of 4.4 at 8,199 rows)
    # the direction columns are data: the native path leaves their gradient zero
    errs = [rel_l2(xn[:, :76], xt[:, :76])] + [rel_l2(a, b) for a, b in zip(gn, gt)]
    print("rel L2 dx_pos, params:", ["%.2e" % e for e in errs])
    assert max(errs) <= 1e-3, errs
