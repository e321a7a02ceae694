"""Are the GPU's reference-numerics gradients different from the oracle's by more than a
summation order? (r05 diagnostic of the N = 1,024 PSNR drift; needs the GPU.)

Trains the reference-semantics oracle (acc="f64", the PSNR test's reference) along the
PSNR test's trajectory (tests/ingp_psnr.py batches and draws, 1,024 samples, 64 rays per
step). At each checkpoint step c, from the oracle's parameters at that step, the step's
gradients are computed three ways on the same batch and draws:
  f64  -- the oracle as trained;
  f32  -- the oracle's f32-accumulation arm (oracle/ref_ingp.py acc="f32"): the spread a
          summation order alone causes;
  gpu  -- the pipeline in reference numerics with the same parameters copied in.
Per module: relative L2 to f64, and the count of entries whose zero / sign pattern differs
from f64 (AdamW with eps = 1e-15 turns those into full lr steps).

    python tools/r5/grad_arms_diag.py [--checkpoints 0,16,32,48] [--out gpurun_out/x.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402


def compare(g, r):
    den = r.norm().clamp_min(1e-300)
    return {"rel_l2": float((g - r).norm() / den),
            "zero_mismatch": int(((g == 0) != (r == 0)).sum()),
            "sign_mismatch": int(((g > 0) & (r < 0)).sum() + ((g < 0) & (r > 0)).sum()),
            "nonzero_ref": int((r != 0).sum()), "n": int(r.numel()),
            "equal_frac": float((g == r).double().mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--checkpoints", default="0,16,32,48")
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/grad_arms.json")
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
    pp = scene.get_point_preprocessor("horizontal")
    p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5,
                           numerics="reference")
    p.send_tensors_to(dev)
    state0 = p.state_dict()
    opt_cfg = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    gopt = p.get_optimizer(opt_cfg)  # zero_grad only

    def oracle(acc):
        return ref_ingp.RefInstantNGP(cfg, state0, ref_ingp.prep_kwargs(pp), p.scale,
                                      scene.max_i, half=True, semantics="reference", acc=acc)

    o64 = oracle("f64")
    o32 = oracle("f32")
    opt = o64.optimizer(opt_cfg)
    cps = sorted(int(c) for c in a.checkpoints.split(","))
    gen = torch.Generator().manual_seed(ingp_psnr.SEED_U)
    loader = BatchLoader(scene, a.batch, seed=ingp_psnr.SEED_BATCH)
    batches = iter(loader)
    rows = []
    for it in range(max(cps) + 1):
        try:
            b = next(batches)
        except StopIteration:
            batches = iter(loader)
            b = next(batches)
        u = torch.rand(b["origin"].shape[0], a.samples, generator=gen)
        cb = ref_ingp.cpu_batch(b)
        if it in cps:
            row = {"iteration": it}
            # f32 arm from the same parameters
            with torch.no_grad():
                for m in ref_ingp.MODULES:
                    o32.params[m].copy_(o64.params[m])
                    o32.params[m].grad = None
            r32 = o32.forward(cb, u)
            o32.loss(cb, r32).backward()
            # GPU from the same parameters
            with torch.no_grad():
                for m in ref_ingp.MODULES:
                    getattr(p, m).params.copy_(o64.params[m].detach().float())
            gopt.zero_grad()
            rg = p.forward(b, u=u.to(dev))
            lg = p.compute_loss(b, rg)
            lg.backward()
            torch.cuda.synchronize()
        r64 = o64.forward(cb, u)
        l64 = o64.loss(cb, r64)
        opt.zero_grad()
        l64.backward()
        if it in cps:
            row["loss"] = {"f64": float(l64), "f32": float(o32.loss(cb, r32).detach()),
                           "gpu": float(lg)}
            cm64 = r64["color_map_fine"].detach().double()
            row["color_map"] = {
                "f32": compare(r32["color_map_fine"].detach().double(), cm64),
                "gpu": compare(rg["color_map_fine"].detach().double().cpu(), cm64)}
            for m in ref_ingp.MODULES:
                g64 = o64.params[m].grad.detach()
                row[m] = {"f32": compare(o32.params[m].grad.detach(), g64),
                          "gpu": compare(getattr(p, m).params.grad.detach().double().cpu(), g64)}
            rows.append(row)
            print(json.dumps(row), flush=True)
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "w") as f:
                json.dump(rows, f, indent=1)
        opt.step()


if __name__ == "__main__":
    main()
