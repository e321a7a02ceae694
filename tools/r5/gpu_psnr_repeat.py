"""Run-to-run spread of the GPU pipeline in reference numerics (GPU only, no oracle).

Trains R copies of the pipeline of tests/test_ingp_oracle_gpu.py::
test_psnr_vs_reference_semantics (same scene, seed-5 parameters, batches and draws) side by
side and prints their PSNR at the test's checkpoints. The hash grid backward sums with f32
atomics whose order varies from run to run (as tinycudann's do), so the copies separate the
way two reference runs would; that spread sits beside the oracle's own
(tools/ingp_oracle_spread.py --scene-device cuda).

    python tools/r5/gpu_psnr_repeat.py --samples 1024 --batch 64 --runs 4
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402

from tests import ingp_psnr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--checkpoints", default="0,8,32,48,64")
    ap.add_argument("--numerics", default="reference")
    ap.add_argument("--out", default=None)
    ap.add_argument("--with-build", action="store_true",
                    help="also train a build-numerics pipeline interleaved (as the test does)")
    ap.add_argument("--no-surface-stream", action="store_true",
                    help="the surface branch on the main stream")
    ap.add_argument("--with-oracle", action="store_true",
                    help="also train the reference-semantics oracle interleaved (as the test)")
    a = ap.parse_args()
    import __graft_entry__ as ge
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    dev = torch.device("cuda")
    opt = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
    cfg = ge._ingp_config(a.samples)
    runners = {}
    for r in range(a.runs):
        p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5,
                               numerics=a.numerics)
        if a.no_surface_stream:
            p.surface_stream = False
        p.send_tensors_to(dev)
        runners[f"gpu_run{r}"] = ingp_psnr.PipelineRunner(p, opt, dev)
        if r == 0 and a.with_build:
            pb = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5)
            pb.send_tensors_to(dev)
            runners["gpu_build"] = ingp_psnr.PipelineRunner(pb, opt, dev)
        if r == 0 and a.with_oracle:
            from oracle import ref_ingp
            pp = scene.get_point_preprocessor("horizontal")
            o = ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp), p.scale,
                                       scene.max_i, half=True, semantics="reference")
            runners["oracle"] = ingp_psnr.OracleRunner(o, opt)
    cps = tuple(int(c) for c in a.checkpoints.split(","))

    def progress(out):
        it = next(iter(out.values()))[-1]["iteration"]
        print("checkpoint", it, {k: round(v[-1]["psnr"], 4) for k, v in out.items()},
              flush=True)

    res = ingp_psnr.train_side_by_side(runners, scene, a.samples, checkpoints=cps,
                                       batch=a.batch, progress=progress)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
