"""Train Instant-NGP on the synthetic scene's volume-truth mode and score its extinction
against the ground truth (SURVEY §8 d: trained / extracted extinction vs a known field).

    python tools/volume_truth_score.py [--views 16] [--img 96] [--iters 2000] [--out f.json]

The scene's radiance is rendered through a known extinction field
(datasets/synthetic.py, radiance_model="volume"); training runs the product pipeline
(the same kernels as bench.py) with AdamW; at checkpoints the extract path
(atmonr_amd.extract: the loop of scripts/extract.py:180-211) evaluates the extinction on
the pixel grid x altitudes, and the score is the Pearson r and the scale-fitted relative
L2 error against SyntheticHARP2Dataset.extinction_truth at the same points, plus the
image PSNR (harp2.py:310-335). Prints one JSON object (and writes it with --out).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=16)
    ap.add_argument("--img", type=int, default=96)
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--truth-samples", type=int, default=512)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--checkpoints", default="0,250,500,1000,2000")
    ap.add_argument("--alt-step", type=float, default=500.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)

    import __graft_entry__ as ge
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.extract import GridExtractDataset, extract_volume
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from tests.ingp_psnr import render_psnr

    t0 = time.time()
    scene = SyntheticHARP2Dataset(n_views=args.views, img_size=args.img, device=dev, seed=0,
                                  radiance_model="volume", truth_samples=args.truth_samples)
    t_scene = time.time() - t0
    cfg = ge._ingp_config(args.samples)
    pipe = InstantNGPPipeline(cfg, scene)
    pipe.send_tensors_to(dev)
    opt_cfg = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-6}
    opt = pipe.get_optimizer(opt_cfg)
    grid = GridExtractDataset(scene, alt_step=args.alt_step)
    checkpoints = sorted(int(c) for c in args.checkpoints.split(","))
    record = {"scene": {"views": args.views, "img": args.img, "rays": len(scene),
                        "truth_samples": args.truth_samples, "build_s": round(t_scene, 2)},
              "train": {"samples_per_ray": args.samples, "batch": args.batch,
                        "optimizer": {"AdamW": opt_cfg}},
              "extract_grid": {"points": len(grid), "alt_step_m": args.alt_step},
              "checkpoints": []}

    def score(it, loss):
        pipe.eval()
        sigma = extract_volume(pipe, scene, grid)
        pipe.train()
        alt = grid.sample_alt[None, None].expand_as(grid.lat)
        s = scene.score_extinction(sigma[:, 0], grid.lat.reshape(-1), grid.lon.reshape(-1),
                                   alt.reshape(-1))
        # column (vertically summed) extinction per pixel: where the clouds are, whatever
        # height the fit puts them at
        A = grid.sample_alt.shape[0]
        col_p = sigma[:, 0].double().view(*grid.shp, A).sum(-1)
        col_t = scene.extinction_truth(grid.lat.double(), grid.lon.double(),
                                       alt.double()).sum(-1)
        pc, tc = col_p - col_p.mean(), col_t - col_t.mean()
        s["column_pearson_r"] = float((pc * tc).sum() / (pc.norm() * tc.norm()))
        psnr = render_psnr(lambda b, u: pipe.forward(b, u=u.to(dev))["color_map_fine"],
                           scene, args.samples)
        row = {"iteration": it, "loss": loss, "psnr": psnr, **s}
        record["checkpoints"].append(row)
        print(json.dumps(row), flush=True)

    loader = BatchLoader(scene, args.batch, seed=3)
    batches = iter(loader)
    loss = float("nan")
    for it in range(args.iters + 1):
        if it in checkpoints:
            score(it, loss)
        if it == args.iters:
            break
        try:
            b = next(batches)
        except StopIteration:
            batches = iter(loader)
            b = next(batches)
        lo = pipe.compute_loss(b, pipe.forward(b))
        opt.zero_grad()
        lo.backward()
        opt.step()
        loss = float(lo.detach())
    print(json.dumps(record))
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(record, f, indent=1)


if __name__ == "__main__":
    main()
