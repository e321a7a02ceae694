"""Which side of the N = 1,024 reference-numerics PSNR drift is systematic: the GPU's
gradients or the GPU's optimizer? (diagnostic of tests/test_ingp_oracle_gpu.py
test_psnr_vs_reference_semantics[1024-...]; needs the GPU)

Trains, on the test's batches and draws, side by side:
  oracle  -- the reference-semantics oracle with its f64 torch AdamW (the test's reference);
  gpu     -- the pipeline in reference numerics with FusedAdam (what the test checks);
  hybrid  -- the oracle's parameters and AdamW, but each step's gradients computed by the
             GPU pipeline from those same parameters (copied in before the step).
If `hybrid` tracks `oracle`, the per-step gradients agree and the drift comes from the
optimizer / parameter storage; if it drifts like `gpu`, from the gradients.

    python tools/psnr_hybrid_diag.py [--iters 64] [--every 8] [--out gpurun_out/hybrid.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402


class HybridRunner:
    def __init__(self, pipe, oracle, opt_cfg, dev):
        from oracle import ref_ingp

        self.p, self.o, self.dev = pipe, oracle, dev
        self.gopt = pipe.get_optimizer(opt_cfg)  # zero_grad only, never stepped
        self.opt = oracle.optimizer(opt_cfg)
        self.modules = ref_ingp.MODULES

    def _load(self):
        with torch.no_grad():
            for m in self.modules:
                getattr(self.p, m).params.copy_(self.o.params[m].detach().float())

    def step(self, b, u, it):
        self._load()
        loss = self.p.compute_loss(b, self.p.forward(b, u=u.to(self.dev)))
        self.gopt.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
        self.opt.zero_grad()
        for m in self.modules:
            g = getattr(self.p, m).params.grad
            self.o.params[m].grad = g.detach().double().cpu().clone()
        self.opt.step()
        return loss.item()

    def render(self, b, u):
        from oracle import ref_ingp

        return self.o.forward(ref_ingp.cpu_batch(b), u)["color_map_fine"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--every", type=int, default=8)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/psnr_hybrid.json")
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
    pp = scene.get_point_preprocessor("horizontal")

    def pipe():
        p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5,
                               numerics="reference")
        p.send_tensors_to(dev)
        return p

    p_gpu, p_hyb = pipe(), pipe()

    def oracle():
        return ref_ingp.RefInstantNGP(cfg, p_gpu.state_dict(), ref_ingp.prep_kwargs(pp),
                                      p_gpu.scale, scene.max_i, half=True,
                                      semantics="reference")

    opt = {"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}
    runners = {"oracle": ingp_psnr.OracleRunner(oracle(), opt),
               "gpu": ingp_psnr.PipelineRunner(p_gpu, opt, dev),
               "hybrid": HybridRunner(p_hyb, oracle(), opt, dev)}
    rows = []

    def record(out):
        row = {"iteration": out["oracle"][-1]["iteration"]}
        for k in runners:
            row["psnr_" + k] = out[k][-1]["psnr"]
        row["delta_gpu_db"] = row["psnr_gpu"] - row["psnr_oracle"]
        row["delta_hybrid_db"] = row["psnr_hybrid"] - row["psnr_oracle"]
        ro, rh = runners["oracle"].o, runners["hybrid"].o
        for m in ref_ingp.MODULES:
            r = ro.params[m].detach()
            den = r.norm().clamp_min(1e-300)
            row["hyb_param_rel_" + m] = ((rh.params[m].detach() - r).norm() / den).item()
            g = getattr(p_gpu, m).params.detach().double().cpu()
            row["gpu_param_rel_" + m] = ((g - r).norm() / den).item()
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
