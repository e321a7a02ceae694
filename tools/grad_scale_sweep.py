"""Per-module f16 gradient error of the fused field backward (build numerics) against the
f64-exact gradient, for several per-wavefront gradient-scale targets
(anr_ingp_field_set_grad_scale: max |dL/dout| of a wavefront -> 2^t). GPU diagnostic.

    python tools/grad_scale_sweep.py [--targets 6 8 10 12] [--samples 64 --rays 200]
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
    ap.add_argument("--targets", type=int, nargs="+", default=[4, 6, 8, 10, 12])
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--rays", type=int, default=200)
    a = ap.parse_args()
    import __graft_entry__ as ge
    from atmonr_amd import _lib
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_ingp

    dev = torch.device("cuda:0")
    torch.set_num_threads(16)
    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
    cfg = ge._ingp_config(a.samples)
    pp = scene.get_point_preprocessor("horizontal")
    B, N = a.rays, a.samples
    batch = next(iter(BatchLoader(scene, B, seed=1)))
    u = torch.rand(B, N, generator=torch.Generator().manual_seed(2))
    cb = ref_ingp.cpu_batch(batch)
    p0 = InstantNGPPipeline(cfg, scene, fused=True, seed=5)
    state = {m: {k: v.clone() for k, v in sd.items()} for m, sd in p0.state_dict().items()}
    exact = ref_ingp.RefInstantNGP(cfg, state, ref_ingp.prep_kwargs(pp), p0.scale, scene.max_i,
                                   half=True, composite="f64")
    exact.loss(cb, exact.forward(cb, u)).backward()
    ref = ref_ingp.RefInstantNGP(cfg, state, ref_ingp.prep_kwargs(pp), p0.scale, scene.max_i,
                                 half=True, semantics="reference")
    ref.loss(cb, ref.forward(cb, u)).backward()
    out = {"reference_semantics": {m: float((ref.params[m].grad - exact.params[m].grad).norm()
                                            / exact.params[m].grad.norm())
                                   for m in ref_ingp.MODULES}}
    lib = _lib.load()
    for t in a.targets:
        prev = lib.anr_ingp_field_set_grad_scale(t)
        p = InstantNGPPipeline(cfg, scene, fused=True, seed=5)
        p.send_tensors_to(dev)
        p.compute_loss(batch, p.forward(batch, u=u.to(dev))).backward()
        torch.cuda.synchronize()
        lib.anr_ingp_field_set_grad_scale(prev)
        out[f"target_2^{t}"] = {m: float((getattr(p, m).params.grad.double().cpu()
                                          - exact.params[m].grad).norm()
                                         / exact.params[m].grad.norm())
                                for m in ref_ingp.MODULES}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
