"""Is the bench's network alive? Per step: loss, fraction of samples with sigma > 0 and
color > 0, fraction of nonzero hash-table gradient entries and of nonzero dL/denc (bench.py's setup: configs[2],
AdamW lr 1e-2, B = 8192, N = 1024 unless overridden)."""

from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--variant", default="baseline")
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--numerics", default="build", choices=["build", "reference"])
    ap.add_argument("--switch-at", type=int, default=0,
                    help="train in build numerics up to this step, then continue from those "
                         "parameters in --numerics (a fresh optimizer)")
    args = ap.parse_args()
    import bench
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.parallel import FlatGradBucket
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline

    dev = torch.device("cuda", 0)
    ds = SyntheticHARP2Dataset(n_views=90, img_size=512, device=dev, seed=0)
    cfg = bench.ingp_config(args.variant, args.samples)
    dt = {"f16": torch.float16, "bf16": torch.bfloat16, "f32": torch.float32}[args.dtype]
    ocfg = {"lr": args.lr, "betas": [0.9, 0.99], "eps": 1e-15, "weight_decay": 1e-2}

    def make(numerics, state=None):
        p = InstantNGPPipeline(cfg, ds, dtype=dt, fused=True, seed=1337, numerics=numerics)
        p.send_tensors_to(dev)
        if state is not None:
            p.load_state_dict(state)
        p._keep_d_enc = True  # dL/denc of each step (field.py diagnostics hook)
        o = p.get_optimizer(ocfg)
        b = FlatGradBucket([q for g in o.param_groups for q in g["params"]], dev)
        return p, o, b, p.pos_encoder.parameters().__next__()

    pipe, opt, bucket, tab = make("build" if args.switch_at else args.numerics)
    loader = BatchLoader(ds, args.batch, shuffle=True, seed=0)
    it = iter(loader)
    for k in range(args.steps):
        if args.switch_at and k == args.switch_at:
            pipe, opt, bucket, tab = make(args.numerics, pipe.state_dict())
            print(f"-- switched to {args.numerics} numerics", flush=True)
        batch = next(it)
        res = pipe.forward(batch)
        loss = pipe.compute_loss(batch, res)
        bucket.zero()
        loss.backward()
        gz = (tab.grad != 0).float().mean().item()
        dz = (pipe._last_d_enc != 0).float().mean().item()
        dr = (pipe._last_d_enc != 0).any(1).float().mean().item()
        sig = res["sigma_fine"]
        col = res["color_fine"]
        print(f"step {k:3d} loss {loss.item():.5f} sigma>0 {(sig > 0).float().mean().item():.4f} "
              f"color>0 {(col > 0).float().mean().item():.4f} table-grad nonzero {gz:.4f} "
              f"dL/denc nonzero {dz:.4f} rows {dr:.4f} "
              f"pred mean {res['color_map_fine'].float().mean().item():.4f} "
              f"target mean {batch['rad'].float().mean().item():.4f}", flush=True)
        opt.step()


if __name__ == "__main__":
    main()
