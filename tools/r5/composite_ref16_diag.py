"""The reference-numerics composite backward on the pipeline's own inputs (r05 PSNR-drift
diagnostic; needs the GPU): the oracle's f16 colour / density / surface colour and z of
the PSNR test's first step (1,024 samples, 64 rays) through oracle/ref_f16 (torch-CUDA
restatement) and through the GPU kernel (anr_composite_ref16_*), with the same dL/dC.
Prints where dL/dsigma and dL/dcolor differ and the inputs around those samples.

    python tools/r5/composite_ref16_diag.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import __graft_entry__ as ge
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.graphics_utils import render_with_surface_ref16
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_f16, ref_ingp
    from tests import ingp_psnr

    torch.set_num_threads(16)
    dev = torch.device("cuda:0")
    N, B = 1024, 64
    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
    cfg = ge._ingp_config(N)
    p = InstantNGPPipeline(cfg, scene, dtype=torch.float16, fused=True, seed=5,
                           numerics="reference")
    pp = scene.get_point_preprocessor("horizontal")
    o = ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp), p.scale,
                               scene.max_i, half=True, semantics="reference")
    gen = torch.Generator().manual_seed(ingp_psnr.SEED_U)
    b = next(iter(BatchLoader(scene, B, seed=ingp_psnr.SEED_BATCH)))
    u = torch.rand(B, N, generator=gen)
    cb = ref_ingp.cpu_batch(b)
    cap = {}
    orig = ref_f16.render_with_surface

    def spy(z_km, color, sigma, color_surf, acc="cuda"):
        cap.update(z_km=z_km.detach().clone(), color=color.detach().half(),
                   sigma=sigma.detach().half(), cs=color_surf.detach().half())
        return orig(z_km, color, sigma, color_surf, acc)
    ref_f16.render_with_surface = spy
    res = o.forward(cb, u)
    ref_f16.render_with_surface = orig
    loss = o.loss(cb, res)
    (g_cm,) = torch.autograd.grad(loss, res["color_map_fine"])
    g_cm = g_cm.half()
    # oracle composite alone, same inputs and dL/dC
    col = cap["color"].clone().requires_grad_(True)
    sig = cap["sigma"].clone().requires_grad_(True)
    cs = cap["cs"].clone().requires_grad_(True)
    cm_o = ref_f16.render_with_surface(cap["z_km"], col, sig, cs)[0]
    cm_o.backward(g_cm)
    # GPU composite, z in the pipeline's units with z_scale (as the pipeline calls it)
    from oracle import ref_path
    _, z = ref_path.sample_uniform_bins(cb["origin"], cb["dir"], cb["len"], u=u, n_bins=N)
    print("z dtype", z.dtype, "z_km equal to z*scale/1000 in f32:",
          torch.equal((z.float() * np.float32(p.scale / 1000)), cap["z_km"].float()), flush=True)
    colg = cap["color"].float().to(dev).requires_grad_(True)
    sigg = cap["sigma"].float().to(dev).requires_grad_(True)
    csg = cap["cs"].float().to(dev).requires_grad_(True)
    cm_g = render_with_surface_ref16(z.float().to(dev), colg, sigg, csg,
                                     z_scale=p.scale / 1000)[0]
    cm_g.backward(g_cm.to(dev).to(cm_g.dtype))
    print("color_map equal:", torch.equal(cm_g.detach().cpu().half(), cm_o.detach().half()))
    for name, a, gpu in (("sigma", sig.grad, sigg.grad), ("color", col.grad, colg.grad),
                         ("color_surf", cs.grad, csg.grad)):
        a = a.double().reshape(-1)
        g = gpu.detach().double().cpu().reshape(-1)
        diff = a != g
        print(f"d_{name}: differ {int(diff.sum())} of {a.numel()}, rel_l2 "
              f"{float((a - g).norm() / a.norm().clamp_min(1e-30)):.3e}", flush=True)
        if name == "sigma" and diff.any():
            rays = sorted({int(i) // N for i in torch.nonzero(diff).view(-1).tolist()})
            np.savez(os.path.join(ROOT, "gpurun_out", "r5_comp_rays.npz"), rays=np.array(rays),
                     z_km=cap["z_km"][rays].numpy(), color=cap["color"][rays].float().numpy(),
                     sigma=cap["sigma"][rays].float().numpy(), cs=cap["cs"][rays].float().numpy(),
                     g_cm=g_cm[rays].float().numpy(),
                     ds_oracle=a.view(-1, N)[rays].numpy(), ds_gpu=g.view(-1, N)[rays].numpy())
            idx = torch.nonzero(diff).view(-1)[:8].tolist()
            zk = cap["z_km"].half().double().reshape(-1)
            sg = cap["sigma"].double().reshape(-1)
            for i in idx:
                r_, s_ = divmod(i, N)
                lo, hi = max(0, s_ - 2), min(N, s_ + 3)
                print(f"  ray {r_} sample {s_}: oracle {a[i]:.6e} gpu {g[i]:.6e}; "
                      f"z_km16 {zk[r_ * N + lo:r_ * N + hi].tolist()} "
                      f"sigma {sg[r_ * N + lo:r_ * N + hi].tolist()}", flush=True)


if __name__ == "__main__":
    main()
