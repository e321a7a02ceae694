"""Run-to-run spread of the GPU pipeline itself at the N = 1,024 PSNR test's shape (needs
the GPU). Trains the reference-numerics pipeline K times from the same seed on the test's
batches and draws (tests/ingp_psnr.py) and prints PSNR per checkpoint per run. The f32
atomics of the hash-grid and field backward sum in a different order on every run, so
runs differ by rounding; this measures how far that alone moves PSNR. Also writes, for the
first step, the per-entry comparison of the hash-grid gradient with the oracle's
(relative L2, sign flips and how many entries differ by one f16 quantum).

    python tools/psnr_gpu_self_spread.py [--runs 3] [--out gpurun_out/self_spread.json]
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
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--checkpoints", default="0,8,16,32,48,64")
    ap.add_argument("--numerics", default="reference")
    ap.add_argument("--out", default="gpurun_out/psnr_self_spread.json")
    a = ap.parse_args()
    import __graft_entry__ as ge
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_ingp
    from tests import ingp_psnr

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    dev = torch.device("cuda:0")
    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
    cfg = ge._ingp_config(a.samples)
    opt = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    rec = {}

    def pipe():
        p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5,
                               numerics=a.numerics)
        p.send_tensors_to(dev)
        return p

    # step-0 gradient of the hash grid, GPU vs oracle, entry by entry
    p = pipe()
    pp = scene.get_point_preprocessor("horizontal")
    o = ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp), p.scale,
                               scene.max_i, half=True, semantics="reference")
    b = next(iter(BatchLoader(scene, a.batch, seed=ingp_psnr.SEED_BATCH)))
    u = torch.rand(b["origin"].shape[0], a.samples,
                   generator=torch.Generator().manual_seed(ingp_psnr.SEED_U))
    p.compute_loss(b, p.forward(b, u=u.to(dev))).backward()
    cb = ref_ingp.cpu_batch(b)
    o.loss(cb, o.forward(cb, u)).backward()
    for m in ref_ingp.MODULES:
        gg = getattr(p, m).params.grad.detach().double().cpu()
        go = o.params[m].grad.detach()
        nz = (gg != 0) | (go != 0)
        # one quantum: the f16 spacing of g * 128, divided by 128
        q = torch.from_numpy(__import__("numpy").spacing(
            (go.abs() * 128).clamp_min(2.0 ** -24).half().float().numpy()
            .astype("float16")).astype("float64")) / 128
        d = (gg - go).abs() / q
        rec[f"step0_{m}"] = {
            "nonzero": int(nz.sum()), "equal": int(((gg == go) & nz).sum()),
            "differ_1q": int(((d > 0.5) & (d < 1.5) & nz).sum()),
            "differ_gt1q": int(((d >= 1.5) & nz).sum()),
            "sign_flips": int(((gg.sign() * go.sign()) < 0).sum()),
            "zero_mismatch": int(((gg == 0) != (go == 0)).sum()),
            "rel_l2": ((gg - go).norm() / go.norm().clamp_min(1e-300)).item(),
            "small_nonzero_lt4q": int(((go.abs() < 4 * q) & (go != 0)).sum())}
        print(m, rec[f"step0_{m}"], flush=True)
    del p, o
    cps = tuple(int(c) for c in a.checkpoints.split(","))
    runs = {f"run{k}": ingp_psnr.PipelineRunner(pipe(), opt, dev) for k in range(a.runs)}
    out = ingp_psnr.train_side_by_side(runs, scene, a.samples, checkpoints=cps, batch=a.batch)
    for k, v in out.items():
        print(k, [round(r["psnr"], 4) for r in v], flush=True)
    rec["psnr"] = out
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
