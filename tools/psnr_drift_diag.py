"""Where the reference-numerics pipeline and the reference-semantics oracle drift apart at
1,024 samples per ray (diagnostic of tests/test_ingp_oracle_gpu.py
test_psnr_vs_reference_semantics[1024-...]; needs the GPU).

Trains both side by side exactly as the test does (8-view 16x16 scene built on the GPU,
batch 64, the test's batches and draws) and records, every --every iterations, both PSNRs,
both losses and the relative L2 distance of every module's parameters (GPU vs oracle).
One JSON to --out.

    python tools/psnr_drift_diag.py [--iters 64] [--every 8] [--out gpurun_out/drift.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--every", type=int, default=8)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/psnr_drift.json")
    a = ap.parse_args()
    import __graft_entry__ as ge
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_ingp
    from tests import ingp_psnr

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    dev = torch.device("cuda:0")
    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
    cfg = ge._ingp_config(a.samples)
    p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5,
                           numerics="reference")
    p.send_tensors_to(dev)
    pp = scene.get_point_preprocessor("horizontal")
    o = ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp), p.scale,
                               scene.max_i, half=True, semantics="reference")
    opt = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    runners = {"gpu": ingp_psnr.PipelineRunner(p, opt, dev),
               "oracle": ingp_psnr.OracleRunner(o, opt)}
    rows = []

    def record(out):
        it = out["gpu"][-1]["iteration"]
        row = {"iteration": it}
        for k in runners:
            row["psnr_" + k] = out[k][-1]["psnr"]
            row["loss_" + k] = out[k][-1]["loss"]
        row["delta_db"] = row["psnr_gpu"] - row["psnr_oracle"]
        for m in ref_ingp.MODULES:
            g = getattr(p, m).params.detach().double().cpu()
            r = o.params[m].detach()
            row["param_rel_" + m] = ((g - r).norm() / r.norm().clamp_min(1e-300)).item()
        rows.append(row)
        print(json.dumps(row), flush=True)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)

    cps = tuple(range(0, a.iters + 1, a.every))
    ingp_psnr.train_side_by_side(runners, scene, a.samples, checkpoints=cps, batch=a.batch,
                                 progress=record)


if __name__ == "__main__":
    main()
