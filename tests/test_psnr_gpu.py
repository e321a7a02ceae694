"""PSNR at fixed iterations, GPU path vs the oracle (SURVEY §8 d).

The NeRF pipeline (configs/nerf.json shapes) trains on an 8-view 16x16 synthetic scene on
the GPU and, side by side, the oracle's CPU restatement of the same step (oracle/ref_nerf.py
+ ref_path.py) from the same initial weights, the same batches and the same stratified /
pdf draws; density noise is off in both (it is the only other random input). After 0 and K
iterations every ray is rendered with midpoint samples and the image PSNR of harp2.py:310-335
(atmonr_amd.metrics) is computed for both.

The reference's own NeRF training is chaotic with respect to rounding: the coarse network's
gradient through sample_pdf's t_in_bin (samplers.py:92-96) divides by the cdf width of the
bin a fine sample lands in, so a perturbation of the coarse weights by one f32 rounding
(1e-7 relative) moves the coarse gradient by ~4 % (measured on the oracle alone). Hence two
checks:
* strict: that gradient path detached in both runs (everything else identical), over
  PERMS summation orders per side (hidden units permuted: same mathematics) — the mean
  PSNR after 16 Adam steps within 0.1 dB, every pair's last-batch loss within 5 % (7+ dB
  of training progress);
* reference semantics (path attached): the GPU run must land within the spread of oracle
  runs whose fine-sampler weights are perturbed by one f32 rounding.
With ANR_PSNR_OUT set, the numbers are written there as JSON (profiles/ records them).
"""

import json
import os

import pytest
import torch
import torch.nn.functional as F

from oracle import ref_nerf, ref_path

pytestmark = pytest.mark.gpu

CFG = {"type": "NeRF", "include_height": False, "point_preprocessor": "horizontal",
       "num_bands": 4, "ray_origin_height": 20000, "sampler": {"N_c": 64, "N_f": 128},
       "encoder": {"L_x": [14, 14, 10], "L_d": 4}, "mlp_hidden_dim": 256}


# 8 views x 16 x 16 = 2,048 rays, batches of 128: KS[-1] = 16 steps is one epoch. Sized so
# that each oracle run (CPU, f32) takes ~15 s on 8-16 host threads.
IMG, BATCH, KS = 16, 128, [0, 16]


def _prep_kwargs(pp):
    return dict(scale=float(pp.scale), offset=torch.tensor(pp.offset, dtype=torch.float64),
                lat_min=pp.lat_min, lat_range=pp.lat_range, lon_min=pp.lon_min,
                lon_range=pp.lon_range, h0=pp.ray_origin_height, shift_lon=pp.shift_lon)


class _Oracle:
    """nerf.py:73-240 with explicit draws (oracle functions), Adam as nerf.py:56-71."""

    def __init__(self, sd, pp, scale, lr):
        self.nets = {}
        for mode, V in (("coarse", 1), ("fine", 4)):
            n = ref_nerf.RefAtmoNeRF(76, 24, 4, V, CFG["mlp_hidden_dim"])
            n.load_state_dict({k: v.detach().cpu() for k, v in sd[mode].items()})
            n.eval()  # density noise off (the pipeline side runs in eval mode too)
            self.nets[mode] = n
        self.prep, self.scale = _prep_kwargs(pp), scale
        params = [p for m in ("coarse", "fine") for p in self.nets[m].parameters()]
        self.opt = torch.optim.Adam(params, lr=lr)

    def _stage(self, mode, b, u, w_c=None, z_c=None):
        B = b["origin"].shape[0]
        if mode == "coarse":
            N = 64
            bins = torch.linspace(0, 1, N + 1)[None]
            z = (bins[:, :-1] + u / N) * b["len"][:, None]
            pts = b["origin"][:, None] + b["dir"][:, None] * z[..., None]
        else:
            N = 192
            pts, z = ref_nerf.sample_pdf(b["origin"], b["dir"], w_c, z_c, 128, u=u)
        pts = ref_nerf.preprocess_torch(pts, **self.prep)
        pe = ref_path.positional_encoding(pts, [14, 14, 10]).view(B * N, -1)
        de = ref_path.positional_encoding(b["dir"][:, None].repeat(1, N, 1), 4).view(B * N, -1)
        color, sigma = self.nets[mode](torch.cat([pe, de], dim=1))
        color = torch.exp(torch.clamp(color.view(B, N, -1), max=11))
        sigma = F.relu(sigma.view(B, N, -1))
        cm, _, w = ref_path.render(z * (self.scale / 1000), color, sigma)
        return cm, w, z

    def forward(self, b, u_c, u_f):
        cm_c, w_c, z_c = self._stage("coarse", b, u_c)
        cm_f, _, _ = self._stage("fine", b, u_f, w_c, z_c)
        return cm_c, cm_f

    def step(self, b, u_c, u_f):
        cm_c, cm_f = self.forward(b, u_c, u_f)
        idx = b["irgb_idx"][:, None]
        loss = (F.mse_loss(torch.take_along_dim(cm_c, idx, 1)[:, 0], b["rad"])
                + F.mse_loss(torch.take_along_dim(cm_f, idx, 1)[:, 0], b["rad"]))
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.item()


def _render_all(fwd, scene, chunk=1024):
    """Fine colour of every ray at the observed band, midpoint draws (u = 0.5)."""
    n = len(scene)
    out = torch.empty(n)
    with torch.no_grad():
        for s in range(0, n, chunk):
            idx = torch.arange(s, min(n, s + chunk), device=scene.device)
            b = scene.__getbatch__(idx)
            B = idx.numel()
            cm_f = fwd(b, torch.full((B, 64), 0.5), torch.full((B, 128), 0.5))
            out[s:s + B] = torch.take_along_dim(cm_f.float().cpu(), b["irgb_idx"].cpu()[:, None], 1)[:, 0]
    return out


def _setup(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    scene = SyntheticHARP2Dataset(n_views=8, img_size=IMG, device=dev, seed=0)
    # NeRF colours are exp(sigmoid(.)) in (1, e): targets rescaled into that range
    scene.ray_rad = scene.ray_rad * (2.5 / scene.max_i)
    scene.max_i = 2.5
    return scene


def permute_hidden(sd: dict, seed: int) -> dict:
    """An AtmoNeRF state dict with the hidden units of every layer (fc1-fc8's 256, fc9's
    first 256, fc10's 128) permuted, and the next layer's input columns with them: the
    same network to the last bit of its exact arithmetic, with every dot product summed
    in another order. Adam is elementwise, so training is permutation-equivariant too: a
    permutation arm samples the run-to-run freedom of the GEMM summation order (as two
    BLAS libraries differ) without changing the mathematics."""
    g = torch.Generator().manual_seed(seed)
    sd = {k: v.detach().clone() for k, v in sd.items()}
    h = sd["fc1.weight"].shape[0]
    for i in range(1, 11):
        n_hidden = h if i <= 9 else sd["fc10.weight"].shape[0]
        p = torch.randperm(n_hidden, generator=g).to(sd[f"fc{i}.weight"].device)
        full = torch.arange(sd[f"fc{i}.weight"].shape[0], device=p.device)
        full[:n_hidden] = p  # fc9's density rows stay in place
        sd[f"fc{i}.weight"] = sd[f"fc{i}.weight"][full]
        sd[f"fc{i}.bias"] = sd[f"fc{i}.bias"][full]
        nxt = {9: 10, 10: 11}.get(i, i + 1)
        w = sd[f"fc{nxt}.weight"]
        cols = torch.arange(w.shape[1], device=p.device)
        cols[:n_hidden] = p  # fc6's skip and fc10's direction columns stay in place
        sd[f"fc{nxt}.weight"] = w[:, cols]
    return sd


def _train(dev, scene, K, gpu, detach_pdf, perturb_seed=None, lr=5e-4, permute_seed=None):
    """Train either the GPU pipeline or the oracle from the same init (seed 0) on the same
    batches and draws; return [(iteration, loss, PSNR)] at the iterations in K.
    ``permute_seed``: both networks' hidden units permuted first (permute_hidden)."""
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.pipelines.factory import get_pipeline
    import atmonr_amd.pipelines.nerf as nmod

    torch.manual_seed(0)
    pipe = get_pipeline(CFG, scene)
    pipe.send_tensors_to(dev)
    if permute_seed is not None:
        pipe.load_state_dict({m: permute_hidden(s, 1000 * permute_seed + j)
                              for j, (m, s) in enumerate(pipe.state_dict().items())})
    pipe.eval()  # density noise off
    pp = scene.get_point_preprocessor("horizontal")
    orig_dev, orig_ref = nmod.sample_pdf, ref_nerf.sample_pdf
    pert = torch.Generator().manual_seed(perturb_seed or 0)

    def dev_pdf(rb, w, z, n_samples=128, u=None):
        if perturb_seed is not None:  # the same one-rounding perturbation on the GPU side
            n = 1e-7 * torch.randn(w.shape, generator=pert)
            w = w + (w * n.to(w.device)).detach()
        return orig_dev(rb, w.detach() if detach_pdf else w, z, n_samples=n_samples, u=u)

    def ref_pdf(o, d, w, z, n, u=None):
        if perturb_seed is not None:  # one f32 rounding of the weights, gradient unchanged
            w = w + (w * (1e-7 * torch.randn(w.shape, generator=pert)) ).detach()
        return orig_ref(o, d, w.detach() if detach_pdf else w, z, n, u=u)

    nmod.sample_pdf, ref_nerf.sample_pdf = dev_pdf, ref_pdf
    try:
        if gpu:
            opt = pipe.get_optimizer({"lr": lr})
            fwd = lambda b, uc, uf: pipe.forward(b, u_coarse=uc.to(dev), u_fine=uf.to(dev))["color_map_fine"]

            def step(b, uc, uf):
                res = pipe.forward(b, u_coarse=uc.to(dev), u_fine=uf.to(dev))
                loss = pipe.compute_loss(b, res)
                opt.zero_grad()
                loss.backward()
                opt.step()
                return loss.item()
        else:
            orc = _Oracle(pipe.state_dict(), pp, pipe.scale, lr)
            fwd = lambda b, uc, uf: orc.forward({k: v.cpu() for k, v in b.items()}, uc, uf)[1]
            step = lambda b, uc, uf: orc.step({k: v.cpu() for k, v in b.items()}, uc, uf)
        target = scene.target_image()
        gen = torch.Generator().manual_seed(7)
        batches = iter(BatchLoader(scene, BATCH, seed=3))
        out, it, loss = [], 0, float("nan")
        for k in K:
            while it < k:
                b = next(batches)
                B = b["origin"].shape[0]
                uc, uf = torch.rand(B, 64, generator=gen), torch.rand(B, 128, generator=gen)
                loss = step(b, uc, uf)
                it += 1
            pix = _render_all(fwd, scene)
            psnr = scene.get_image_metrics(scene.scatter_image(pix.to(dev)), target)["PSNR_mean"]
            out.append((it, loss, psnr))
        return out
    finally:
        nmod.sample_pdf, ref_nerf.sample_pdf = orig_dev, orig_ref


_REC = {}


def _dump():
    out = os.environ.get("ANR_PSNR_OUT")
    if out:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as f:
            json.dump(_REC, f, indent=1)


# CPU oracle training dominates these tests (minutes on a GPU box's host share): the
# per-test limit is raised above the suite's --timeout.
PERMS = 8


@pytest.mark.timeout(900)
def test_psnr_at_fixed_iterations_strict(dev):
    """t_in_bin gradient detached in both. A NeRF run at this scale is itself a draw from
    the summation order of its GEMMs: 1e-7 relative perturbations of the pdf weights
    spread one side's 16-iteration PSNR by ~0.12 dB, and so does changing the order in
    which every dot product is summed -- the freedom two BLAS libraries have. The bar
    therefore applies to distributions over that freedom: both sides train PERMS times,
    each time with the hidden units of both networks permuted by the same permutation
    (permute_hidden: the same mathematics, every dot product summed in another order),
    and the mean PSNR over the GPU runs and over the oracle runs must agree within 0.1 dB
    at every checkpoint; each pair's last-batch loss (128 rays) within 5 %. Measured
    (profiles/r06_nerf_psnr_permutations.md): native kernels 15.846, library GEMMs
    15.864, oracle 15.838 dB, while the unpermuted pair alone sits 0.12 dB apart -- one
    draw, not an offset: a native-forward/library-backward hybrid lands with the native
    runs, and both forwards render the same weights to the same PSNR bit for bit."""
    scene = _setup(dev)
    K = KS
    _REC["iterations"] = K
    gpus = [_train(dev, scene, K, gpu=True, detach_pdf=True, permute_seed=p)
            for p in range(PERMS)]
    arms = [_train(dev, scene, K, gpu=False, detach_pdf=True, permute_seed=p)
            for p in range(PERMS)]
    means = [{"iteration": K[i], "gpu_mean": sum(r[i][2] for r in gpus) / PERMS,
              "oracle_mean": sum(a[i][2] for a in arms) / PERMS} for i in range(len(K))]
    for m in means:
        m["delta_means_db"] = m["gpu_mean"] - m["oracle_mean"]
    _REC["strict"] = {"gpu_permutations": gpus, "oracle_permutations": arms, "means": means}
    _dump()
    for i, m in enumerate(means):
        assert abs(m["delta_means_db"]) < 0.1, _REC
        for g, o in zip(gpus, arms):
            if g[i][1] == g[i][1]:  # not NaN (iteration 0 has no loss)
                assert abs(g[i][1] - o[i][1]) < 5e-2 * o[i][1], _REC
    assert means[-1]["gpu_mean"] > means[0]["gpu_mean"] + 1.0, _REC


@pytest.mark.timeout(900)
def test_psnr_at_fixed_iterations_reference_semantics(dev):
    """Reference semantics: within the spread of oracle runs one f32 rounding apart."""
    scene = _setup(dev)
    K = KS
    g = _train(dev, scene, K, gpu=True, detach_pdf=False)
    runs = [_train(dev, scene, K, gpu=False, detach_pdf=False, perturb_seed=s) for s in (1, 2, 3)]
    _REC["full"] = {"gpu": g, "oracle_perturbed": runs}
    _dump()
    ps = [r[-1][2] for r in runs]
    lo, hi = min(ps), max(ps)
    margin = max(0.5, hi - lo)
    assert lo - margin <= g[-1][2] <= hi + margin, _REC
