"""Which NeRF kernel carries the configs[1] PSNR offset?

Runs tests/test_psnr_gpu.py's strict 16-step training (t_in_bin detached) for perturbation
seeds 0..S-1 with the AtmoNeRF layers split between the native kernels
(csrc/nerf_mlp.hip) and torch's library GEMMs:
  native      forward and backward native (the default)
  torch       ANR_NERF_MLP=torch
  nfwd_tbwd   native forward; the backward as torch GEMMs on the native forward's saved
              activations (same chain as _AtmoNeRFFn.backward, masks from y > 0)
and, with --mlp-accuracy, the per-layer gradient of one step's actual MLP inputs for each
arm against an f64 evaluation of the same inputs (relative L2 and the signed projection
<g - g64, g64> / |g64|^2, which shows a systematic scale bias).

    python tools/nerf_hybrid_arms.py --seeds 5 --out gpurun_out/nerf_hybrid.json
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402

from tests import test_psnr_gpu as T  # noqa: E402


def _torch_backward(ctx, dcolor, dsigma):
    """_AtmoNeRFFn.backward's chain with torch ops on the saved native activations."""
    net = ctx.net
    x, *rest = ctx.saved_tensors
    ys, (color, sigma) = rest[:10], rest[10:12]
    h, pc = net.hidden_dim, net.pos_channels
    L = [getattr(net, f"fc{i}") for i in range(1, 12)]
    n9, out = L[8].out_features, L[10].out_features
    y = [None] + [t for t in ys]            # y[i] = output of fc i (padded ld)
    act = {i: y[i][:, :L[i - 1].out_features] for i in range(1, 11)}
    x_pos, x_dir = x[:, :pc], x[:, pc:]
    inputs = {1: x_pos, 6: torch.cat([act[5], x_pos], 1), 9: act[8],
              10: torch.cat([act[9][:, :h], x_dir], 1), 11: act[10]}
    for i in (2, 3, 4, 5, 7, 8):
        inputs[i] = act[i - 1]
    grads = {}
    g = dcolor * (1 - color) * color                            # fc11 pre-activation
    for i in range(11, 0, -1):
        W = L[i - 1].weight
        grads[i] = (g.t() @ inputs[i], g.sum(0))
        if i == 1:
            break
        gin = g @ W                                              # dL/d(input of fc i)
        if i == 10:
            g9 = torch.zeros(g.shape[0], n9, device=g.device)
            g9[:, :h] = gin[:, :h]
            g9[:, h:] = torch.where(sigma > 0, dsigma, torch.zeros_like(dsigma))
            g = g9
        elif i == 6:
            g = gin[:, :h] * (act[5] > 0)
        else:
            g = gin * (act[i - 1] > 0)
    pg = []
    for i in range(1, 12):
        pg += list(grads[i])
    return (None, None, None, *pg)


def _set_arm(arm):
    import atmonr_amd.nerf_model as nm

    if not hasattr(nm._AtmoNeRFFn, "_orig_backward"):
        nm._AtmoNeRFFn._orig_backward = nm._AtmoNeRFFn.backward
    nm._NATIVE = arm != "torch"
    orig = nm._AtmoNeRFFn._orig_backward
    if arm == "nfwd_tbwd":
        nm._AtmoNeRFFn.backward = staticmethod(_torch_backward)
    else:
        nm._AtmoNeRFFn.backward = staticmethod(orig)


def psnr_arms(dev, seeds, arms):
    scene = T._setup(dev)
    rec = {a: {} for a in arms}
    for s in seeds:
        ps = None if s == 0 else s
        for arm in arms:
            if arm == "oracle32":
                _set_arm("native")
                rec[arm][s] = T._train(dev, scene, T.KS, gpu=False, detach_pdf=True,
                                       perturb_seed=ps)
                continue
            _set_arm(arm)
            rec[arm][s] = T._train(dev, scene, T.KS, gpu=True, detach_pdf=True,
                                   perturb_seed=ps)
        _set_arm("native")
        print("seed", s, {a: round(r[s][-1][2], 4) for a, r in rec.items()}, flush=True)
    means = {a: sum(r[s][-1][2] for s in seeds) / len(seeds) for a, r in rec.items()}
    print("mean PSNR at", T.KS[-1], {a: round(m, 4) for a, m in means.items()}, flush=True)
    return {"runs": rec, "mean": means}


def permutation_arms(dev, seeds, arms):
    """The strict test's training with both networks' hidden units permuted
    (tests/test_psnr_gpu.permute_hidden, seed p on every side): the same mathematics with
    every dot product summed in another order. Paired per permutation, a systematic
    native-vs-oracle offset shows in every pair; summation-order chaos averages out."""
    scene = T._setup(dev)
    rec = {a: {} for a in arms}
    for p in seeds:
        for arm in arms:
            _set_arm("native" if arm == "oracle32" else arm)
            rec[arm][p] = T._train(dev, scene, T.KS, gpu=arm != "oracle32", detach_pdf=True,
                                   permute_seed=p)
        _set_arm("native")
        print("permutation", p, {a: round(r[p][-1][2], 4) for a, r in rec.items()}, flush=True)
    means = {a: sum(r[p][-1][2] for p in seeds) / len(seeds) for a, r in rec.items()}
    print("permutation mean PSNR at", T.KS[-1], {a: round(m, 4) for a, m in means.items()},
          flush=True)
    return {"runs": rec, "mean": means}


def render_check(dev, train_arm="torch", seed=0):
    """Train with ``train_arm`` (the strict test's 16 steps), then render every ray of the
    scene with the native and with the library forward from the SAME weights: PSNR of each
    and the largest per-ray colour difference."""
    import atmonr_amd.nerf_model as nm
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.pipelines.factory import get_pipeline

    scene = T._setup(dev)
    _set_arm(train_arm)
    torch.manual_seed(0)
    pipe = get_pipeline(T.CFG, scene)
    pipe.send_tensors_to(dev)
    pipe.eval()
    opt = pipe.get_optimizer({"lr": 5e-4})
    import atmonr_amd.pipelines.nerf as nmod
    orig = nmod.sample_pdf
    nmod.sample_pdf = lambda rb, w, z, n_samples=128, u=None: orig(rb, w.detach(), z,
                                                                     n_samples=n_samples, u=u)
    try:
        gen = torch.Generator().manual_seed(7)
        batches = iter(BatchLoader(scene, T.BATCH, seed=3))
        for _ in range(T.KS[-1]):
            b = next(batches)
            B = b["origin"].shape[0]
            uc, uf = torch.rand(B, 64, generator=gen), torch.rand(B, 128, generator=gen)
            res = pipe.forward(b, u_coarse=uc.to(dev), u_fine=uf.to(dev))
            loss = pipe.compute_loss(b, res)
            opt.zero_grad()
            loss.backward()
            opt.step()
        out = {}
        fwd = lambda b, uc, uf: pipe.forward(b, u_coarse=uc.to(dev), u_fine=uf.to(dev))[
            "color_map_fine"]
        target = scene.target_image()
        for arm in ("native", "torch"):
            nm._NATIVE = arm == "native"
            pix = T._render_all(fwd, scene)
            out[arm] = {"pix": pix, "psnr": float(scene.get_image_metrics(
                scene.scatter_image(pix.to(dev)), target)["PSNR_mean"])}
        nm._NATIVE = True
    finally:
        nmod.sample_pdf = orig
        _set_arm("native")
    d = (out["native"]["pix"] - out["torch"]["pix"]).abs()
    rec = {"trained_with": train_arm, "psnr_native_render": out["native"]["psnr"],
           "psnr_torch_render": out["torch"]["psnr"], "max_abs_pixel_diff": float(d.max()),
           "mean_abs_pixel_diff": float(d.mean())}
    print("render check", rec, flush=True)
    return rec


def mlp_accuracy(dev, n_steps=8):
    """Per-layer MLP gradients of real training inputs: each arm vs f64."""
    import atmonr_amd.nerf_model as nm
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.pipelines.factory import get_pipeline

    scene = T._setup(dev)
    torch.manual_seed(0)
    pipe = get_pipeline(T.CFG, scene)
    pipe.send_tensors_to(dev)
    pipe.eval()
    captured = {}
    orig_fwd = nm.AtmoNeRF.forward

    def spy(self, x, noise=None):
        captured.setdefault(id(self), x.detach().clone())
        return orig_fwd(self, x, noise)

    gen = torch.Generator().manual_seed(7)
    batches = iter(BatchLoader(scene, T.BATCH, seed=3))
    opt = pipe.get_optimizer({"lr": 5e-4})
    out = []
    for it in range(n_steps):
        b = next(batches)
        B = b["origin"].shape[0]
        uc, uf = torch.rand(B, 64, generator=gen), torch.rand(B, 128, generator=gen)
        captured.clear()
        nm.AtmoNeRF.forward = spy
        try:
            res = pipe.forward(b, u_coarse=uc.to(dev), u_fine=uf.to(dev))
        finally:
            nm.AtmoNeRF.forward = orig_fwd
        loss = pipe.compute_loss(b, res)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if it not in (0, n_steps - 1):
            continue
        for mode in ("coarse", "fine"):
            net = pipe.nerf[mode]
            x = captured[id(net)]
            tg = torch.Generator(device=dev).manual_seed(11)
            gcol = gsig = None
            rows = {}
            for arm in ("native", "torch", "f64"):
                nm._NATIVE = arm == "native"
                if arm == "f64":
                    ref = nm.AtmoNeRF(net.pos_channels, net.dir_channels, net.out_channels,
                                      net.volume_channels, net.hidden_dim).to(dev).double()
                    ref.load_state_dict({k: v.double() for k, v in net.state_dict().items()})
                    ref.eval()
                    m, xi = ref, x.double()
                else:
                    m, xi = net, x
                m.zero_grad(set_to_none=True)
                color, sigma = m(xi)
                if gcol is None:  # one upstream gradient for every arm
                    gcol = torch.randn(color.shape, generator=tg, device=dev)
                    gsig = torch.randn(sigma.shape, generator=tg, device=dev)
                torch.autograd.backward([color, sigma], [gcol.to(color.dtype),
                                                         gsig.to(sigma.dtype)])
                rows[arm] = ({k: p.grad.detach().double().clone()
                              for k, p in m.named_parameters()},
                             color.detach().double(), sigma.detach().double())
                nm._NATIVE = True
            r64 = rows["f64"][0]
            rec = {"iteration": it, "mode": mode, "rows": x.shape[0], "arms": {}}
            for arm in ("native", "torch"):
                g = rows[arm][0]
                rec["arms"][arm] = {
                    "color_rel": float((rows[arm][1] - rows["f64"][1]).norm()
                                       / rows["f64"][1].norm()),
                    "sigma_rel": float((rows[arm][2] - rows["f64"][2]).norm()
                                       / max(float(rows["f64"][2].norm()), 1e-300)),
                    "grad_rel": {k: float((g[k] - r64[k]).norm() / r64[k].norm()) for k in r64},
                    "grad_proj": {k: float(((g[k] - r64[k]) * r64[k]).sum() / (r64[k] ** 2).sum())
                                  for k in r64}}
            out.append(rec)
            print(f"iteration {it} {mode}: colour rel native "
                  f"{rec['arms']['native']['color_rel']:.2e} torch "
                  f"{rec['arms']['torch']['color_rel']:.2e}", flush=True)
            for k in r64:
                n, t = rec["arms"]["native"], rec["arms"]["torch"]
                print(f"  {k:12s} rel native {n['grad_rel'][k]:.2e} torch {t['grad_rel'][k]:.2e}"
                      f" | proj native {n['grad_proj'][k]:+.2e} torch {t['grad_proj'][k]:+.2e}",
                      flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--arms", default="native,torch,nfwd_tbwd,oracle32")
    ap.add_argument("--mlp-accuracy", action="store_true")
    ap.add_argument("--render-check", action="store_true")
    ap.add_argument("--perms", type=int, default=0)
    ap.add_argument("--perm-arms", default="native,torch,oracle32")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    if a.mlp_accuracy:
        res["mlp_accuracy"] = mlp_accuracy(dev)
    if a.render_check:
        res["render_check"] = [render_check(dev, arm) for arm in ("torch", "native")]
    if a.seeds:
        res["psnr"] = psnr_arms(dev, range(a.seeds), a.arms.split(","))
    if a.perms:
        res["permutations"] = permutation_arms(dev, range(a.perms), a.perm_arms.split(","))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
