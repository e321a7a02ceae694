"""Does the reference's own arithmetic kill the density field on the bench scene? (CPU only)

ADVICE r04: the reference-numerics headline is timed from a build-numerics warm start
because the GPU's reference numerics leave a dead density field from a cold start
(sigma > 0 at 0 %, dL/denc all zero; profiles/r04_liveness_reference.log). This trains the
reference-semantics ORACLE (oracle/ref_ingp.py, f64 masters, the reference's f16 roundings)
from the same cold start on the bench scene and config (BASELINE configs[2]: 90-view
512x512 synthetic HARP2 scene, T = 2^19, 1,024 samples per ray, AdamW lr 1e-2, seed-1337
parameters) at a reduced batch, and prints per step the fraction of samples with sigma > 0
and of nonzero dL/d(hash table) -- the quantities tools/liveness.py prints for the GPU.

    python tools/r5/oracle_liveness.py --batch 256 --steps 6
"""

from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402

from oracle import ref_ingp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--semantics", default="reference")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    import bench
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    t0 = time.time()
    ds = SyntheticHARP2Dataset(n_views=90, img_size=512, device=torch.device("cpu"), seed=0)
    cfg = bench.ingp_config("baseline", a.samples)
    p = InstantNGPPipeline(cfg, ds, dtype=torch.float16, fused=True, seed=1337)
    pp = ds.get_point_preprocessor("horizontal")
    o = ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp), p.scale, ds.max_i,
                               half=True, semantics=a.semantics)
    opt = o.optimizer({"lr": 1e-2, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2})
    loader = BatchLoader(ds, a.batch, shuffle=True, seed=0)
    gen = torch.Generator().manual_seed(0)
    it = iter(loader)
    print(f"scene + oracle ready in {time.time() - t0:.0f}s; batch {a.batch} x {a.samples}",
          flush=True)
    for k in range(a.steps):
        b = ref_ingp.cpu_batch(next(it))
        u = torch.rand(b["origin"].shape[0], a.samples, generator=gen)
        res = o.forward(b, u)
        loss = o.loss(b, res)
        opt.zero_grad()
        loss.backward()
        sig = res["sigma_fine"]
        g = o.params["pos_encoder"].grad
        gz = (g != 0).double().mean().item() if g is not None else 0.0
        print(f"step {k:2d} loss {loss.item():.5f} sigma>0 {(sig > 0).double().mean().item():.4f} "
              f"table-grad nonzero {gz:.4f}  ({time.time() - t0:.0f}s)", flush=True)
        opt.step()


if __name__ == "__main__":
    main()
