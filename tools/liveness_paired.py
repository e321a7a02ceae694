"""Cold-start liveness, paired: the GPU pipeline in reference numerics beside the
reference-semantics oracle with f64 masters and with f32 masters.

All runners start from the same seed-1337 parameters of BASELINE configs[2] (T = 2^19,
1,024 samples per ray, AdamW lr 1e-2 / wd 1e-2 / eps 1e-15) on the bench scene (90-view
512x512 synthetic HARP2, built on the GPU as bench.py builds it), and every step feeds them
the same batch and the same stratified draws. Per step and runner it prints the loss and
the fraction of fine samples with sigma > 0. tinycudann's torch binding keeps f32 master
parameters, and so do the GPU's FusedAdam and the f32-master arm (parameters and AdamW
moments rounded to f32 after every step, tests/ingp_psnr.OracleRunner master="f32"); the
oracle's default arm keeps f64 masters.

The revival step is the first step from which sigma > 0 stays above --alive (default 0.5).

    python tools/liveness_paired.py --batch 128 --steps 30 --out gpurun_out/live_b128.json
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

OPT = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}


def revival(trace, alive):
    """collapse_step: the first step with sigma>0 below 0.1 (None: never collapsed);
    revival_step: after the collapse, the first step from which sigma>0 stays above
    ``alive`` to the end (None: not revived within the run)."""
    fr = [t["sigma_pos"] for t in trace]
    col = next((k for k, f in enumerate(fr) if f < 0.1), None)
    rev = None
    if col is not None:
        for k in range(len(fr) - 1, col, -1):
            if fr[k] <= alive:
                break
            rev = k
    return {"collapse_step": col, "revival_step": rev}


def run(batch, steps, samples, numerics, arms, threads, scene_img, views):
    import bench
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_ingp
    from tests.ingp_psnr import OracleRunner

    torch.set_num_threads(threads)
    dev = torch.device("cuda", 0)
    t0 = time.time()
    ds = SyntheticHARP2Dataset(n_views=views, img_size=scene_img, device=dev, seed=0)
    cfg = bench.ingp_config("baseline", samples)
    p = InstantNGPPipeline(cfg, ds, dtype=torch.float16, fused=True, seed=1337,
                           numerics=numerics)
    p.send_tensors_to(dev)
    state = {m: {k: v.detach().clone() for k, v in sd.items()}
             for m, sd in p.state_dict().items()}
    opt = p.get_optimizer(OPT)
    pp = ds.get_point_preprocessor("horizontal")
    oracles = {}
    for name in arms:
        master = {"oracle_f64_master": "f64", "oracle_f32_master": "f32"}[name]
        o = ref_ingp.RefInstantNGP(cfg, state, ref_ingp.prep_kwargs(pp), p.scale, ds.max_i,
                                   half=True, semantics="reference" if numerics == "reference"
                                   else "build")
        oracles[name] = OracleRunner(o, OPT, master=master)
    loader = BatchLoader(ds, batch, shuffle=True, seed=0)
    gen = torch.Generator().manual_seed(0)
    it = iter(loader)
    trace = {"gpu": [], **{k: [] for k in oracles}}
    print(f"scene + runners ready in {time.time() - t0:.0f}s; batch {batch} x {samples}, "
          f"{numerics} numerics", flush=True)
    for k in range(steps):
        b = next(it)
        u = torch.rand(b["origin"].shape[0], samples, generator=gen)
        res = p.forward(b, u=u.to(dev))
        sig = res["sigma_fine"]
        loss = p.compute_loss(b, res)
        opt.zero_grad()
        loss.backward()
        opt.step()
        trace["gpu"].append({"loss": float(loss), "sigma_pos": float((sig > 0).float().mean())})
        for name, r in oracles.items():
            oloss = r.step(b, u, k)
            ores = r.last
            trace[name].append({"loss": float(oloss),
                                "sigma_pos": float((ores["sigma_fine"] > 0).double().mean())})
        print(f"step {k:2d} " + "  ".join(
            f"{n} loss {t[-1]['loss']:.5f} sigma>0 {t[-1]['sigma_pos']:.4f}"
            for n, t in trace.items()) + f"  ({time.time() - t0:.0f}s)", flush=True)
    return trace


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--numerics", default="reference", choices=["reference", "build"])
    ap.add_argument("--arms", default="oracle_f64_master,oracle_f32_master")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--alive", type=float, default=0.5)
    ap.add_argument("--img-size", type=int, default=512)
    ap.add_argument("--views", type=int, default=90)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    trace = run(a.batch, a.steps, a.samples, a.numerics, [x for x in a.arms.split(",") if x],
                a.threads, a.img_size, a.views)
    summary = {k: revival(t, a.alive) for k, t in trace.items()}
    print("summary", json.dumps(summary), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"args": vars(a), "trace": trace, "summary": summary}, f, indent=1)


if __name__ == "__main__":
    main()
