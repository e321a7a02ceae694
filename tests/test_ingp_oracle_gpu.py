"""Instant-NGP train step and PSNR at fixed iterations: GPU pipeline vs the oracle.

The oracle (oracle/ref_ingp.py) restates instant_ngp.py:137-263 in float64 torch on the
CPU with autograd, over the restated tcnn modules (ref_tcnn: tcnn semantics, unpinned
against real tinycudann). Same initial parameters (the pipeline's state_dict), same rays
and the same stratified draws on both sides.

* step parity, f32 modules (the exact-f32 kernels): color maps within 1e-4 of the
  largest value, loss within 1e-5 relative, z bit-exact, every module's parameter
  gradient within 2e-3 relative L2 error (measured: 2e-6, 3e-7, 3e-6; dir MLP 7e-4);
* step parity, f16 modules (the bench configuration: f16 tables / weights, fused field
  kernels) against the oracle with the same f16 roundings (``half=True``): color maps
  within 2e-2, loss within 5e-3 relative, gradients within 1e-1 relative L2 error (the
  fused backward carries f16 gradient tiles the oracle keeps in f64; measured on MI355X:
  color maps 3e-4, loss 2e-6, hash table 1.5e-2, dir MLP 4.4e-2, others <= 1.3e-3);
* the same step at BASELINE configs[2]'s 1,024 samples per ray (24 rays, 24,576 samples:
  f32 and f16), same tolerances;
* PSNR at fixed iterations (SURVEY §8 d): the f16 pipeline and the half-rounding oracle
  train side by side for one epoch (8 AdamW steps, configs/instant_ngp.json optimizer)
  on an 8-view 16x16 scene; the full-image PSNR (harp2.py:310-335) of a midpoint render
  must agree within 0.1 dB at 0 and 8 iterations.
* step parity in REFERENCE NUMERICS (InstantNGPPipeline(numerics="reference"): the
  reference's f16 composite and loss op by op, tcnn's x128 loss-scaled f16 backward,
  f16 parameter gradients) against the oracle's reference semantics (oracle/ref_ingp.py
  semantics="reference", composite / loss from oracle/ref_f16.py with torch's CUDA
  accumulation), at 64 and 1,024 samples per ray: color maps within 1e-2, loss 5e-3,
  gradients 1e-3 relative L2 (measured: colour maps, loss and the dir / surface
  gradients bit-exact, hash table 2.4e-5, pos MLP 8e-5);
* f16 gradient error anchored to tcnn semantics: per module, the relative L2 distance
  to the f64-exact gradient of the same f16-rounded forward, for the GPU build
  numerics, the GPU reference numerics and the oracle's reference semantics; the build's
  must not exceed the reference's own;
* PSNR against reference semantics: the pipeline in reference numerics, the pipeline in
  build numerics and the reference-semantics oracle train side by side for 64 AdamW
  steps (8 epochs, same batches and draws); PSNR at 0 / 8 / 16 / 32 / 64 iterations, and at
  1,024 samples per ray (64 rays per step) at 0 / 8 / 32 / 48 / 64. The reference-numerics
  pipeline must stay within 0.1 dB of the oracle at EVERY checkpoint (north-star bar);
  past 32 iterations at 1,024 samples, where one run is a draw from a ~0.3 dB spread on
  either side, the nearest pair of the GPU's 4 runs from identical inputs and the
  oracle's 3 arms within 0.1 dB (CHAOS_AFTER); the build numerics' distance is recorded
  beside it.
With ANR_INGP_PSNR_OUT set, the measured errors and PSNRs are written there as JSON.
"""

import json
import os

import pytest
import torch

import __graft_entry__ as ge
from oracle import ref_ingp

pytestmark = pytest.mark.gpu

IMG, BATCH, N, KS = 16, 256, 64, [0, 8]   # 8 views x 16 x 16 = 2,048 rays = 8 batches
OPT = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
# about 3x the largest error measured on MI355X (profiles/r03_ingp_oracle_records.json:
# f32 out 2e-6 / grad 5e-6 apart from the dir MLP's f32-composite noise, which the 4x
# oracle-noise floor below covers; f16 out 3.3e-4 / loss 8e-6 / grad 7.4e-3 (hash table);
# bf16 grad 2.1e-3; reference numerics out / loss bit-exact, grad 8.2e-5)
TOL = {"f32": {"out": 1e-5, "loss": 1e-6, "grad": 3e-5},
       "f16": {"out": 1e-3, "loss": 3e-5, "grad": 2.5e-2},
       # bf16 field MLPs (8 significant bits, unscaled bf16 gradient tiles) over f16 tables
       "bf16": {"out": 1e-3, "loss": 3e-5, "grad": 1e-2},
       # reference numerics vs reference semantics: the composite / loss are bit-exact
       # restatements (test_ref16_gpu.py); what differs is the f16 MLPs' accumulation
       # order (MFMA f32 vs the oracle's f64 then f16) and the hash gradient's summation
       "ref16": {"out": 1e-5, "loss": 1e-5, "grad": 3e-4}}
_REC = {}


def _dump():
    out = os.environ.get("ANR_INGP_PSNR_OUT")
    if out:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as f:
            json.dump(_REC, f, indent=1)


@pytest.fixture(scope="module")
def scene(dev):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    return SyntheticHARP2Dataset(n_views=8, img_size=IMG, device=dev, seed=0)


def _pair(scene, dev, dtype, mlp_dtype=None, n_samples=N, oracle_only=None,
          composite="f32", numerics="build"):
    """(GPU pipeline, oracle from its initial parameters); with ``oracle_only`` = an
    existing pipeline, just another oracle of it (``composite`` "f32" or "f64").
    numerics="reference": the pipeline in reference numerics and the oracle in reference
    semantics (the reference's f16 composite / loss / loss-scaled tcnn backward)."""
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    cfg = ge._ingp_config(n_samples)
    p = oracle_only
    if p is None:
        p = InstantNGPPipeline(cfg, scene, dtype=dtype, fused=True, seed=5, mlp_dtype=mlp_dtype,
                               numerics=numerics)
        p.send_tensors_to(dev)
    dtype = p.pos_encoder.dtype
    mlp_dtype = p.pos_mlp.dtype
    pp = scene.get_point_preprocessor("horizontal")
    state = p.state_dict() if oracle_only is None else p._anr_initial_state
    o = ref_ingp.RefInstantNGP(cfg, state, ref_ingp.prep_kwargs(pp), p.scale,
                               scene.max_i, half=dtype == torch.float16,
                               mlp_half="bf16" if mlp_dtype == torch.bfloat16 else None,
                               composite=composite,
                               semantics="reference" if numerics == "reference" else "build")
    if oracle_only is None:
        p._anr_initial_state = {m: {k: v.detach().clone() for k, v in sd.items()}
                                for m, sd in p.state_dict().items()}
        return p, o
    return o


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("prec,n_samples,B", [("f32", N, 200), ("f16", N, 200),
                                              ("bf16", N, 200),
                                              # BASELINE configs[2]'s 1024 samples per ray
                                              ("f32", 1024, 24), ("f16", 1024, 24)])
def test_train_step_matches_oracle(scene, dev, prec, n_samples, B):
    from atmonr_amd.batch_loader import BatchLoader

    p, o = _pair(scene, dev, torch.float32 if prec == "f32" else torch.float16,
                 torch.bfloat16 if prec == "bf16" else None, n_samples)
    batch = next(iter(BatchLoader(scene, B, seed=1)))
    u = torch.rand(B, n_samples, generator=torch.Generator().manual_seed(2))
    res = p.forward(batch, u=u.to(dev))
    loss = p.compute_loss(batch, res)
    loss.backward()
    cb = ref_ingp.cpu_batch(batch)
    ro = o.forward(cb, u)
    lo = o.loss(cb, ro)
    lo.backward()
    tol = TOL[prec]
    rec = {"loss_gpu": loss.item(), "loss_oracle": lo.item()}
    assert torch.equal(res["z_vals_fine"].cpu(), ro["z_vals_fine"])  # sampler bit-exact
    # color maps against the largest rendered value (atmo + surf = color_map); the
    # per-sample fields against their own largest value (recorded, not asserted)
    cmax = ro["color_map_fine"].detach().abs().max()
    for k in ("color_map_fine", "color_map_atmo", "color_map_surf", "color_fine",
              "sigma_fine", "color_surf"):
        x, y = res[k].detach().double().cpu(), ro[k].detach().double()
        scale = cmax if k.startswith("color_map") else y.abs().max()
        rec[k] = ((x - y).abs().max() / scale).item()
    rec["loss_rel"] = abs(loss.item() - lo.item()) / abs(lo.item())
    # the oracle's own f32 noise: the same step with an exact (f64) composite. The dir
    # MLP's gradient sums dL/dcolor over every sample of a ray, and at 1,024 samples the
    # f32 transmittance products move it by 3e-3 (4e-4 at 64): the GPU's f32 composite,
    # evaluated in another order, may differ from the oracle's by a few times that
    o64 = _pair(scene, dev, None, None, n_samples, oracle_only=p, composite="f64")
    ro64 = o64.forward(cb, u)
    o64.loss(cb, ro64).backward()
    for m in ref_ingp.MODULES:
        g = getattr(p, m).params.grad.double().cpu()
        rec["grad_" + m] = _rel(g, o.params[m].grad)
        rec["grad_" + m + "_vs_f64_composite"] = _rel(g, o64.params[m].grad)
        rec["oracle_f32_noise_" + m] = _rel(o.params[m].grad, o64.params[m].grad)
    _REC["step_" + prec + ("" if n_samples == N else f"_n{n_samples}")] = rec
    _dump()
    for k in ("color_map_fine", "color_map_atmo", "color_map_surf"):
        assert rec[k] <= tol["out"], (k, rec)
    assert rec["loss_rel"] <= tol["loss"], rec
    for m in ref_ingp.MODULES:
        bar = max(tol["grad"], 4 * rec["oracle_f32_noise_" + m])
        assert rec["grad_" + m] <= bar, (m, bar, rec)


def _render_psnr(fwd, scene, dev, chunk=1024):
    """Full-image PSNR (harp2.py:310-335) of a midpoint (u = 0.5) render of every ray."""
    n = len(scene)
    pix = torch.empty(n)
    with torch.no_grad():
        for s in range(0, n, chunk):
            idx = torch.arange(s, min(n, s + chunk), device=scene.device)
            b = scene.__getbatch__(idx)
            cm = fwd(b, torch.full((idx.numel(), N), 0.5))
            pix[s:s + idx.numel()] = torch.take_along_dim(
                cm.double().cpu(), b["irgb_idx"].cpu()[:, None], 1)[:, 0].float()
    img = scene.scatter_image(pix.to(dev))
    return scene.get_image_metrics(img, scene.target_image())["PSNR_mean"]


@pytest.mark.timeout(900)
def test_psnr_at_fixed_iterations_matches_oracle(scene, dev):
    from atmonr_amd.batch_loader import BatchLoader

    p, o = _pair(scene, dev, torch.float16)
    opt_g, opt_o = p.get_optimizer(OPT), o.optimizer(OPT)

    def fwd_g(b, u):
        return p.forward(b, u=u.to(dev))["color_map_fine"]

    def fwd_o(b, u):
        return o.forward(ref_ingp.cpu_batch(b), u)["color_map_fine"]

    gen = torch.Generator().manual_seed(7)
    batches = iter(BatchLoader(scene, BATCH, seed=3))
    out, it = [], 0
    for k in KS:
        lg = lo = float("nan")
        while it < k:
            b = next(batches)
            u = torch.rand(b["origin"].shape[0], N, generator=gen)
            lg_t = p.compute_loss(b, p.forward(b, u=u.to(dev)))
            opt_g.zero_grad()
            lg_t.backward()
            opt_g.step()
            cb = ref_ingp.cpu_batch(b)
            lo_t = o.loss(cb, o.forward(cb, u))
            opt_o.zero_grad()
            lo_t.backward()
            opt_o.step()
            lg, lo, it = lg_t.item(), lo_t.item(), it + 1
        out.append({"iteration": it, "loss_gpu": lg, "loss_oracle": lo,
                    "psnr_gpu": _render_psnr(fwd_g, scene, dev),
                    "psnr_oracle": _render_psnr(fwd_o, scene, dev)})
    _REC["psnr"] = out
    _dump()
    for r in out:
        assert abs(r["psnr_gpu"] - r["psnr_oracle"]) < 0.1, out
    assert out[-1]["psnr_gpu"] > out[0]["psnr_gpu"] + 0.5, out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_samples,B", [(N, 200), (1024, 24)])
def test_train_step_reference_numerics(scene, dev, n_samples, B):
    """numerics="reference" (the reference's f16 composite / loss and tcnn's loss-scaled
    f16 backward, csrc/ref16.hip + anr_ingp_field_bwd_ref16) against the oracle's
    reference semantics, same parameters, rays and draws."""
    from atmonr_amd.batch_loader import BatchLoader

    p, o = _pair(scene, dev, torch.float16, n_samples=n_samples, numerics="reference")
    batch = next(iter(BatchLoader(scene, B, seed=1)))
    u = torch.rand(B, n_samples, generator=torch.Generator().manual_seed(2))
    res = p.forward(batch, u=u.to(dev))
    loss = p.compute_loss(batch, res)
    loss.backward()
    cb = ref_ingp.cpu_batch(batch)
    ro = o.forward(cb, u)
    lo = o.loss(cb, ro)
    lo.backward()
    rec = {"loss_gpu": loss.item(), "loss_oracle": lo.item(),
           "zero_rays": int(p._zero_rays.item())}
    assert res["color_map_fine"].dtype == torch.float16 and loss.dtype == torch.float16
    assert torch.equal(res["z_vals_fine"].cpu(), ro["z_vals_fine"])
    cmax = ro["color_map_fine"].detach().double().abs().max()
    for k in ("color_map_fine", "color_map_atmo", "color_map_surf"):
        x, y = res[k].detach().double().cpu(), ro[k].detach().double()
        rec[k] = ((x - y).abs().max() / cmax).item()
        rec[k + "_bit_exact_frac"] = (x == y).double().mean().item()
    rec["loss_rel"] = abs(loss.item() - lo.item()) / abs(lo.item())
    for m in ref_ingp.MODULES:
        g = getattr(p, m).params.grad.double().cpu()
        rec["grad_" + m] = _rel(g, o.params[m].grad)
        rec["grad_zero_agree_" + m] = ((g == 0) == (o.params[m].grad == 0)).double().mean().item()
    _REC["step_reference_numerics" + ("" if n_samples == N else f"_n{n_samples}")] = rec
    _dump()
    assert rec["zero_rays"] == 0
    tol = TOL["ref16"]
    for k in ("color_map_fine", "color_map_atmo", "color_map_surf"):
        assert rec[k] <= tol["out"], (k, rec)
    assert rec["loss_rel"] <= tol["loss"], rec
    for m in ref_ingp.MODULES:
        assert rec["grad_" + m] <= tol["grad"], (m, rec)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_samples,B", [(N, 200), (1024, 24)])
def test_f16_gradient_error_vs_tcnn_semantics(scene, dev, n_samples, B):
    """Per-module relative L2 error of the f16 gradients against the f64-exact gradient
    of the same f16-rounded forward (oracle half=True, composite and backward in f64),
    for the GPU's build numerics, the GPU's reference numerics, and the oracle's
    reference semantics (what tcnn + the reference's f16 autograd compute). The build's
    f16 backward (f32 between kernels, per-wavefront gradient scale) must be no less
    accurate than the reference's own f16 gradients for every module at the bench's
    1,024 samples per ray; at 64 samples within 1.25x of it (measured: the hash table
    7.4e-3 vs 6.7e-3 -- both are the f16 rounding of the hidden-gradient tiles, which
    the gradient-scale target does not move, tools/grad_scale_sweep.py -- and every
    other module 5x-80,000x better)."""
    from atmonr_amd.batch_loader import BatchLoader

    p, _ = _pair(scene, dev, torch.float16, n_samples=n_samples)
    exact = _pair(scene, dev, None, None, n_samples, oracle_only=p, composite="f64")
    pr, ref = _pair(scene, dev, torch.float16, n_samples=n_samples, numerics="reference")
    batch = next(iter(BatchLoader(scene, B, seed=1)))
    u = torch.rand(B, n_samples, generator=torch.Generator().manual_seed(2))
    cb = ref_ingp.cpu_batch(batch)
    for pipe in (p, pr):
        pipe.compute_loss(batch, pipe.forward(batch, u=u.to(dev))).backward()
    for o in (exact, ref):
        o.loss(cb, o.forward(cb, u)).backward()
    rec = {}
    for m in ref_ingp.MODULES:
        truth = exact.params[m].grad
        rec[m] = {"gpu_build": _rel(getattr(p, m).params.grad.double().cpu(), truth),
                  "gpu_reference_numerics": _rel(getattr(pr, m).params.grad.double().cpu(),
                                                 truth),
                  "oracle_reference_semantics": _rel(ref.params[m].grad, truth)}
    _REC["f16_grad_error_vs_exact" + ("" if n_samples == N else f"_n{n_samples}")] = rec
    _dump()
    slack = 1.0 if n_samples == 1024 else 1.25
    for m, r in rec.items():
        assert r["gpu_build"] <= r["oracle_reference_semantics"] * slack + 1e-6, (m, rec)
        # reference numerics reproduce the reference semantics' own error
        assert abs(r["gpu_reference_numerics"] - r["oracle_reference_semantics"]) <= \
            0.05 * r["oracle_reference_semantics"] + 1e-5, (m, rec)


class _ReferenceRunner:
    """The oracle in reference semantics, as a tests.ingp_psnr runner."""

    def __init__(self, o):
        from tests.ingp_psnr import OracleRunner

        self.r = OracleRunner(o, OPT)
        self.step, self.render = self.r.step, self.r.render


# Past this many iterations at 1,024 samples per ray (64 rays per step) training is chaotic
# (profiles/r05_psnr_chaos_n1024.md, profiles/r06_psnr_n1024_distribution.md): GPU runs from
# identical inputs -- which differ only in the order of the hash-grid backward's f32 atomic
# adds, as tinycudann's runs do -- spread by ~0.1 dB (sd) at 64 iterations, and a one-ulp
# change of every ray direction moves the oracle by up to 0.25 dB, while through 32
# iterations every one of them agrees within 0.01 dB. Past the horizon one run is one draw,
# on either side, so the bar compares the two distributions' means: REPLICAS GPU runs
# against the oracle's ORACLE_ARMS, reference semantics with f32 master parameters as
# tinycudann's torch binding (and the GPU) keep them -- unperturbed and with every ray
# direction one f32 ulp off under three seeds. (The f64-master oracle of the strict checks
# is recorded beside them; it sits at the top of that distribution at 64 iterations.)
CHAOS_AFTER = {1024: 32}
REPLICAS = 16
ORACLE_ARMS = (("oracle_f32_master", "f32", None), ("oracle_f32_master_dirs0", "f32", 0),
               ("oracle_f32_master_dirs1", "f32", 1), ("oracle_f32_master_dirs2", "f32", 2))


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("n_samples,batch,checkpoints", [
    (N, 256, (0, 8, 16, 32, 64)),
    # BASELINE configs[2]'s 1,024 samples per ray, where the reference's f16 composite
    # underflows hardest: 64 rays per step, 2 epochs of the scene
    (1024, 64, (0, 8, 32, 48, 64))])
def test_psnr_vs_reference_semantics(scene, dev, n_samples, batch, checkpoints):
    """PSNR at fixed iterations: the pipeline in reference numerics, the pipeline in build
    numerics and the oracle in reference semantics train side by side on the same batches
    and draws (tests/ingp_psnr.py), at 64 samples per ray (8 epochs of the 8-view 16x16
    scene) and at the bench's 1,024. The north-star bar, 0.1 dB, holds at every
    checkpoint: at 64 samples per ray and at 1,024 through 32 iterations against the run
    itself. Beyond that (CHAOS_AFTER) one run's PSNR is one draw from a distribution, on
    either side, so the bar applies to the distributions' means: the mean of REPLICAS GPU
    runs from identical inputs (the hash-grid backward's atomics order, as tinycudann's)
    and the mean of the oracle's ORACLE_ARMS (f32 masters, as the reference's) agree
    within 0.1 dB. Both sets, their means and spreads are recorded. The
    build numerics' distance is recorded beside it (a deliberate deviation: DESIGN.md
    §3.1). Training must gain >= 3 dB."""
    from tests.ingp_psnr import PipelineRunner, train_side_by_side

    p_ref, o = _pair(scene, dev, torch.float16, numerics="reference", n_samples=n_samples)
    p_build, _ = _pair(scene, dev, torch.float16, n_samples=n_samples)
    for m in ref_ingp.MODULES:  # same initial parameters (seed 5) for both pipelines
        assert torch.equal(getattr(p_ref, m).params, getattr(p_build, m).params)
    runners = {"gpu_reference_numerics": PipelineRunner(p_ref, OPT, dev),
               "gpu_build": PipelineRunner(p_build, OPT, dev),
               "oracle_reference_semantics": _ReferenceRunner(o)}
    horizon = CHAOS_AFTER.get(n_samples)
    replicas, arms = [], []
    if horizon is not None:
        from tests.ingp_psnr import OracleRunner

        for r in range(1, REPLICAS):
            p_r, _ = _pair(scene, dev, torch.float16, numerics="reference",
                           n_samples=n_samples)
            replicas.append(f"gpu_reference_numerics_replica{r}")
            runners[replicas[-1]] = PipelineRunner(p_r, OPT, dev)
        cfg = ge._ingp_config(n_samples)
        pp = scene.get_point_preprocessor("horizontal")
        for name, master, dirs in ORACLE_ARMS:
            oa = ref_ingp.RefInstantNGP(cfg, p_ref._anr_initial_state, ref_ingp.prep_kwargs(pp),
                                        p_ref.scale, scene.max_i, half=True,
                                        semantics="reference")
            runners[name] = OracleRunner(oa, OPT, perturb_dirs=dirs, master=master)
            runners[name].render_from = horizon + 1  # the arms are compared past the horizon
            arms.append(name)
    key = "psnr_reference_semantics" + ("" if n_samples == N else f"_n{n_samples}")
    out = train_side_by_side(runners, scene, n_samples, checkpoints=checkpoints, batch=batch,
                             progress=lambda r: (_REC.update({key: r}), _dump()))
    rows = []
    for i, r in enumerate(out["oracle_reference_semantics"]):
        row = {"iteration": r["iteration"], "psnr_oracle": r["psnr"],
               "psnr_gpu_reference_numerics": out["gpu_reference_numerics"][i]["psnr"],
               "psnr_gpu_build": out["gpu_build"][i]["psnr"]}
        row["delta_reference_numerics_db"] = row["psnr_gpu_reference_numerics"] - r["psnr"]
        row["delta_build_db"] = row["psnr_gpu_build"] - r["psnr"]
        if replicas and r["iteration"] > horizon:
            runs = [row["psnr_gpu_reference_numerics"]] + [out[k][i]["psnr"] for k in replicas]
            oracles = [out[k][i]["psnr"] for k in arms]
            row["psnr_gpu_replicas"] = runs
            row["psnr_oracle_arms"] = oracles
            row["oracle_arm_names"] = arms
            row["gpu_mean"] = sum(runs) / len(runs)
            row["oracle_mean"] = sum(oracles) / len(oracles)
            row["delta_means_db"] = row["gpu_mean"] - row["oracle_mean"]
            row["replica_spread_db"] = max(runs) - min(runs)
            row["oracle_arm_spread_db"] = max(oracles) - min(oracles)
            row["nearest_pair_db"] = min(abs(u - v) for u in runs for v in oracles)
        rows.append(row)
    _REC[key] = rows
    _REC["zero_rays" + key[len("psnr_reference_semantics"):]] = zr = p_ref.zero_rays_total
    _dump()
    assert zr == 0
    for row in rows:
        if horizon is None or row["iteration"] <= horizon:
            assert abs(row["delta_reference_numerics_db"]) <= 0.1, rows
        else:
            assert abs(row["delta_means_db"]) <= 0.1, rows
    assert rows[-1]["psnr_oracle"] > rows[0]["psnr_oracle"] + 3.0, rows


def test_deferred_grad_quantize_same_update(scene, dev):
    """defer_grad_quantize (bench.py's reference-numerics path): the end-of-backward pass
    leaves the f32 sums in param.grad, and FusedAdam rounds them as tinycudann's f16
    gradients while it reads them. From the same gradients (a copy of one backward's) the
    deferred update equals quantise-then-update bit for bit, in the plain and the
    capturable (device-step) forms. (Two separate backward passes are not compared: their
    f32 atomics sum in different orders.)"""
    from atmonr_amd import _lib
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.optim import FusedAdam
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    import __graft_entry__ as ge

    p = InstantNGPPipeline(ge._ingp_config(N), scene, dtype=torch.float16, fused=True,
                           seed=5, numerics="reference")
    p.send_tensors_to(dev)
    o = p.get_optimizer(OPT)
    p.defer_grad_quantize(o)
    b = next(iter(BatchLoader(scene, 128, seed=4)))
    u = torch.rand(b["origin"].shape[0], N, generator=torch.Generator().manual_seed(6))
    p.compute_loss(b, p.forward(b, u=u.to(dev))).backward()
    torch.cuda.synchronize()
    raw = {m: getattr(p, m).params.grad.clone() for m in ref_ingp.MODULES}
    q = {}
    for m, g in raw.items():
        q[m] = g.clone()
        _lib.call("anr_grad_quantize_f16", q[m].data_ptr(), q[m].numel(), 128.0, _lib.stream(dev))
    torch.cuda.synchronize()
    # the deferred pipeline left the sums unrounded
    assert any(not torch.equal(raw[m], q[m]) for m in raw)
    for capturable in (False, True):
        out = []
        for defer in (False, True):
            ps = [torch.nn.Parameter(getattr(p, m).params.detach().clone()) for m in raw]
            for t, m in zip(ps, raw):
                t.grad = (raw[m] if defer else q[m]).clone()
                if defer:
                    t._anr_grad_quant = 128.0
            opt = FusedAdam([{"params": ps[:1] + ps[3:4], "weight_decay": 0.0},
                             {"params": ps[1:3] + ps[4:], "weight_decay": 1e-2}],
                            lr=1e-2, betas=(0.9, 0.99), eps=1e-15, capturable=capturable)
            for _ in range(2):
                opt.step()
            torch.cuda.synchronize()
            out.append(ps)
        for a_, b_ in zip(*out):
            assert torch.equal(a_, b_)
    with pytest.raises(ValueError):
        p.defer_grad_quantize(torch.optim.AdamW(p.parameters(), lr=1e-3))
