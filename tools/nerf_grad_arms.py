"""NeRF configs[1] gradient arms: native f32 MFMA kernels vs the library GEMMs vs the f32 and
f64 oracle, on the trajectory of tests/test_psnr_gpu.py's strict test.

The f32 oracle trains along the strict test's batches and draws (t_in_bin detached). At each
checkpoint every arm takes the oracle's parameters of that step and computes one gradient of
the same batch with the same draws:
  native   the GPU pipeline on csrc/nerf_mlp.hip (the default)
  torch    the GPU pipeline with ANR_NERF_MLP=torch (hipBLASLt GEMMs)
  oracle32 the CPU oracle in f32 (the reference's arithmetic on torch-CPU)
  oracle64 the same oracle with parameters and inputs in f64
and the relative L2 distance of each arm's per-layer gradient to oracle64 is printed. A
kernel defect shows as one arm far from the other two on some layer.

With --psnr the strict test's 16-step training is repeated for seeds 0..S-1 of the 1e-7
perturbation on three sides (native, torch, oracle32) and the per-seed PSNR is recorded.

    python tools/nerf_grad_arms.py --checkpoints 0,4,8,15 --out gpurun_out/nerf_arms.json
"""

from __future__ import annotations

import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import ref_nerf  # noqa: E402
from tests import test_psnr_gpu as T  # noqa: E402


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def _oracle_grads(orc, b, uc, uf, dtype):
    """One loss.backward() of the oracle at its current parameters (no optimizer step)."""
    nets = orc.nets
    if dtype == torch.float64:
        orc = copy.copy(orc)
        orc.nets = {k: copy.deepcopy(v).double() for k, v in nets.items()}
        b = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
        uc, uf = uc.double(), uf.double()
    for n in orc.nets.values():
        n.zero_grad(set_to_none=True)
    cm_c, cm_f = orc.forward(b, uc, uf)
    idx = b["irgb_idx"][:, None]
    loss = (F.mse_loss(torch.take_along_dim(cm_c, idx, 1)[:, 0], b["rad"])
            + F.mse_loss(torch.take_along_dim(cm_f, idx, 1)[:, 0], b["rad"]))
    loss.backward()
    g = {f"{m}.{k}": p.grad.detach().clone() for m, n in orc.nets.items()
         for k, p in n.named_parameters()}
    return float(loss), g


def _gpu_grads(pipe, sd, b, uc, uf, dev, native):
    import atmonr_amd.nerf_model as nm

    nm._NATIVE = native
    pipe.load_state_dict({m: {k: v.to(dev) for k, v in s.items()} for m, s in sd.items()})
    for m in ("coarse", "fine"):
        pipe.nerf[m].zero_grad(set_to_none=True)
    res = pipe.forward(b, u_coarse=uc.to(dev), u_fine=uf.to(dev))
    loss = pipe.compute_loss(b, res)
    loss.backward()
    torch.cuda.synchronize()
    g = {f"{m}.{k}": p.grad.detach().cpu().clone() for m in ("coarse", "fine")
         for k, p in pipe.nerf[m].named_parameters()}
    nm._NATIVE = True
    return float(loss), g


def grad_arms(dev, checkpoints, lr=5e-4):
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.pipelines.factory import get_pipeline
    import atmonr_amd.pipelines.nerf as nmod

    scene = T._setup(dev)
    torch.manual_seed(0)
    pipe = get_pipeline(T.CFG, scene)
    pipe.send_tensors_to(dev)
    pipe.eval()
    pp = scene.get_point_preprocessor("horizontal")
    orc = T._Oracle(pipe.state_dict(), pp, pipe.scale, lr)
    orig_dev, orig_ref = nmod.sample_pdf, ref_nerf.sample_pdf
    nmod.sample_pdf = lambda rb, w, z, n_samples=128, u=None: orig_dev(
        rb, w.detach(), z, n_samples=n_samples, u=u)
    ref_nerf.sample_pdf = lambda o, d, w, z, n, u=None: orig_ref(o, d, w.detach(), z, n, u=u)
    gen = torch.Generator().manual_seed(7)
    batches = iter(BatchLoader(scene, T.BATCH, seed=3))
    out = []
    try:
        for it in range(max(checkpoints) + 1):
            b = next(batches)
            B = b["origin"].shape[0]
            uc, uf = torch.rand(B, 64, generator=gen), torch.rand(B, 128, generator=gen)
            bc = {k: v.cpu() for k, v in b.items()}
            if it in checkpoints:
                sd = {m: {k: v.detach().clone() for k, v in n.state_dict().items()}
                      for m, n in orc.nets.items()}
                arms = {"oracle64": _oracle_grads(orc, bc, uc, uf, torch.float64),
                        "oracle32": _oracle_grads(orc, bc, uc, uf, torch.float32),
                        "native": _gpu_grads(pipe, sd, b, uc, uf, dev, True),
                        "torch": _gpu_grads(pipe, sd, b, uc, uf, dev, False)}
                ref = arms["oracle64"][1]
                rec = {"iteration": it,
                       "loss": {k: v[0] for k, v in arms.items()},
                       "rel_l2_vs_f64": {a: {n: _rel(g[n], ref[n]) for n in ref}
                                          for a, (_, g) in arms.items() if a != "oracle64"},
                       "native_vs_torch": {n: _rel(arms["native"][1][n], arms["torch"][1][n])
                                           for n in ref}}
                out.append(rec)
                print(f"iteration {it} loss", {k: round(v, 7) for k, v in rec["loss"].items()})
                for n in ref:
                    r = {a: rec["rel_l2_vs_f64"][a][n] for a in ("native", "torch", "oracle32")}
                    print(f"  {n:22s} native {r['native']:.2e} torch {r['torch']:.2e} "
                          f"oracle32 {r['oracle32']:.2e}", flush=True)
            orc.step(bc, uc, uf)
    finally:
        nmod.sample_pdf, ref_nerf.sample_pdf = orig_dev, orig_ref
    return out


def psnr_seeds(dev, seeds):
    import atmonr_amd.nerf_model as nm

    scene = T._setup(dev)
    rec = {"native": {}, "torch": {}, "oracle32": {}}
    for s in seeds:
        ps = None if s == 0 else s
        for arm in ("native", "torch"):
            nm._NATIVE = arm == "native"
            rec[arm][s] = T._train(dev, scene, T.KS, gpu=True, detach_pdf=True, perturb_seed=ps)
        nm._NATIVE = True
        rec["oracle32"][s] = T._train(dev, scene, T.KS, gpu=False, detach_pdf=True,
                                      perturb_seed=ps)
        print("seed", s, {a: round(r[s][-1][2], 4) for a, r in rec.items()}, flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--checkpoints", default="0,4,8,15")
    ap.add_argument("--psnr-seeds", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {"grad_arms": grad_arms(dev, [int(c) for c in a.checkpoints.split(",")])}
    if a.psnr_seeds:
        res["psnr"] = psnr_seeds(dev, range(a.psnr_seeds))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
