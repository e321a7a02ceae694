"""Spread of the reference-semantics Instant-NGP oracle under one f16 rounding (CPU only).

Trains oracle/ref_ingp.RefInstantNGP(semantics="reference") exactly as
tests/test_ingp_oracle_gpu.py::test_psnr_vs_reference_semantics does (8-view 16x16 scene,
batch 256, 64 samples per ray, AdamW of configs/instant_ngp.json, same batches and draws),
once unperturbed and once per perturbation k (tests/ingp_psnr.OracleRunner):
``--perturb grad``: at the first step the f16 loss gradient reaching ray k's rendered
colour is moved by one f16 ulp -- one rounding of the reference's f16 backward done the
other way; ``--perturb dirs``: every ray direction moved by one f32 ulp (seed k) -- the
size of the host-vs-device libm differences of scene construction. Prints the PSNR at
0/8/16/32/64 iterations for every run (JSON with --out).

    python tools/ingp_oracle_spread.py [--runs 3] [--out profiles/r03_ingp_oracle_spread.json]
    python tools/ingp_oracle_spread.py --samples 1024 --batch 64 --checkpoints 0,8,64
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402

from oracle import ref_ingp  # noqa: E402
from tests import ingp_psnr  # noqa: E402


def _progress(out):
    it = next(iter(out.values()))[-1]["iteration"]
    print("checkpoint", it, {k: round(v[-1]["psnr"], 4) for k, v in out.items()}, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--samples", type=int, default=64,
                    help="samples per ray (the PSNR test also runs 1,024 at batch 64)")
    ap.add_argument("--batch", type=int, default=ingp_psnr.BATCH)
    ap.add_argument("--checkpoints", default="0,8,16,32,64")
    ap.add_argument("--noise", type=float, default=3e-5,
                    help="--perturb gradnoise: relative per-step gradient noise")
    ap.add_argument("--out", default=None)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--semantics", default="reference")
    ap.add_argument("--scene-device", default="cpu",
                    help="cuda: build the scene on the GPU exactly as the PSNR test does "
                    "(device libm), so the unperturbed run reproduces the test's oracle")
    ap.add_argument("--ref-acc", default="cuda", help="cuda | cpu (oracle/ref_ingp.py)")
    ap.add_argument("--master", default="f64", help="f64 | f32: master parameters / AdamW "
                    "moments of every run (f32 = tinycudann's torch binding, the GPU's)")
    ap.add_argument("--perturb", default="grad", help="grad: one f16 ulp of one ray's "
                    "loss gradient at step 0; dirs: every ray direction by one f32 ulp; "
                    "f32master: one run with f32 parameters / AdamW moments (the "
                    "reference's) beside the oracle's f64 masters; gradnoise: per-step "
                    "relative gradient noise of --noise; sumnoise: the hash grid gradient "
                    "with --noise x u_f32 x sum|terms| of f32 summation-order noise; "
                    "acc: the f32 and f32rev accumulation arms of oracle/ref_ingp.py")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    import __graft_entry__ as ge
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=torch.device(a.scene_device),
                                  seed=0)
    cfg = ge._ingp_config(a.samples)
    p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5)
    if a.scene_device != "cpu":
        p.send_tensors_to(torch.device(a.scene_device))
    state = p.state_dict()
    pp = scene.get_point_preprocessor("horizontal")
    opt = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    runners = {}
    for run in range(-1, a.runs):
        o = ref_ingp.RefInstantNGP(cfg, state, ref_ingp.prep_kwargs(pp), p.scale, scene.max_i,
                                   half=True, semantics=a.semantics, ref_acc=a.ref_acc)
        if run < 0:
            runners["unperturbed"] = ingp_psnr.OracleRunner(o, opt, master=a.master)
        elif a.perturb == "xnoise":
            runners[f"x_noise{run}"] = ingp_psnr.OracleRunner(
                o, opt, grad_noise=(a.noise, 300 + run, "x"), master=a.master)
        elif a.perturb == "sumnoise":
            runners[f"sum_noise{run}"] = ingp_psnr.OracleRunner(
                o, opt, grad_noise=(a.noise, 200 + run, "sum"), master=a.master)
        elif a.perturb == "gradnoise":
            runners[f"grad_noise{run}"] = ingp_psnr.OracleRunner(
                o, opt, grad_noise=(a.noise, 100 + run), master=a.master)
        elif a.perturb == "acc":
            # equally valid summation orders of the sums before each f16 rounding
            # (oracle/ref_ingp.py acc=): f32 in BLAS order, f32 reversed (f64 = unperturbed)
            arm = ("f32", "f32rev", "f32")[run] if run < 3 else None
            if arm and f"acc_{arm}" not in runners:
                o = ref_ingp.RefInstantNGP(cfg, state, ref_ingp.prep_kwargs(pp), p.scale,
                                           scene.max_i, half=True, semantics=a.semantics,
                                           ref_acc=a.ref_acc, acc=arm)
                runners[f"acc_{arm}"] = ingp_psnr.OracleRunner(o, opt, master=a.master)
        elif a.perturb == "f32master":
            if run == 0:
                runners["f32_master"] = ingp_psnr.OracleRunner(o, opt, master="f32")
        elif a.perturb == "grad":
            runners[f"perturb_ray{run}"] = ingp_psnr.OracleRunner(o, opt, perturb_ray=run,
                                                                     master=a.master)
        else:
            runners[f"perturb_dirs{run}"] = ingp_psnr.OracleRunner(o, opt, perturb_dirs=run,
                                                                      master=a.master)
    t0 = time.time()
    cps = tuple(int(c) for c in a.checkpoints.split(",") if int(c) <= a.iters)
    res = ingp_psnr.train_side_by_side(runners, scene, a.samples, checkpoints=cps,
                                       batch=a.batch, progress=_progress)
    for name, out in res.items():
        print(name, [round(r["psnr"], 4) for r in out], flush=True)
    print(f"{time.time() - t0:.0f}s")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
