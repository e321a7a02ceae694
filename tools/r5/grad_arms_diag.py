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

import numpy as np  # noqa: E402
import torch  # noqa: E402


def compare(g, r):
    den = r.norm().clamp_min(1e-300)
    return {"rel_l2": float((g - r).norm() / den),
            "zero_mismatch": int(((g == 0) != (r == 0)).sum()),
            "sign_mismatch": int(((g > 0) & (r < 0)).sum() + ((g < 0) & (r > 0)).sum()),
            "nonzero_ref": int((r != 0).sum()), "n": int(r.numel()),
            "equal_frac": float((g == r).double().mean())}


def table_detail(g_gpu, g64, g32, offsets, top=8):
    """The largest |gpu - f64| entries of the hash-table gradient: level, value triple."""
    d = (g_gpu - g64).abs()
    idx = torch.topk(d, top).indices
    out = []
    for e in idx.tolist():
        lvl = int(np.searchsorted(offsets * 2, e, side="right") - 1)
        out.append({"entry": e, "level": lvl, "f64": float(g64[e]), "f32": float(g32[e]),
                    "gpu": float(g_gpu[e])})
    return out


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

    from oracle import ref_tcnn

    offsets = ref_tcnn.grid_levels(3, 16, 16, 1.3819, int(cfg["instant_ngp"]["encoding"]["log2_hashmap_size"]))[0]
    captured = {}
    orig = ref_ingp._TcnnCall.apply

    def spy(x, params, fn, *rest):
        y = orig(x, params, fn, *rest)
        for tag, o_ in (("enc", o64), ("enc32", o32)):
            if params is o_.params["pos_encoder"] and y.requires_grad:
                y.retain_grad()
                captured[tag] = y
        if params is o64.params["pos_mlp"] and y.requires_grad:
            y.retain_grad()
            captured["pos_out"] = y
        if params is o64.params["dir_mlp"] and y.requires_grad:
            y.retain_grad()
            captured["dir_out"] = y
        return y
    ref_ingp._TcnnCall.apply = spy
    p._keep_d_enc = True
    o64 = oracle("f64")
    o32 = oracle("f32")
    ref_ingp._TcnnCall.apply = spy
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
            for key in ("sigma_fine", "color_fine"):
                a64 = r64[key].detach().double().reshape(-1)
                row[key] = {"f32": compare(r32[key].detach().double().reshape(-1), a64),
                            "gpu": compare(rg[key].detach().double().cpu().reshape(-1), a64)}
            cm64 = r64["color_map_fine"].detach().double()
            row["color_map"] = {
                "f32": compare(r32["color_map_fine"].detach().double(), cm64),
                "gpu": compare(rg["color_map_fine"].detach().double().cpu(), cm64)}
            for m in ref_ingp.MODULES:
                g64 = o64.params[m].grad.detach()
                row[m] = {"f32": compare(o32.params[m].grad.detach(), g64),
                          "gpu": compare(getattr(p, m).params.grad.detach().double().cpu(), g64)}
            g_gpu = p.pos_encoder.params.grad.detach().double().cpu()
            g64 = o64.params["pos_encoder"].grad.detach()
            row["table_top"] = table_detail(g_gpu, g64, o32.params["pos_encoder"].grad.detach(),
                                            offsets)
            # the sample coordinates the GPU walked vs the oracle's (f64 libm differences
            # of the preprocessor move them by ulps; near a cell face that changes the cell)
            from oracle import ref_path, ref_nerf
            pts, _ = ref_path.sample_uniform_bins(cb["origin"], cb["dir"], cb["len"], u=u,
                                                  n_bins=a.samples)
            pts = (ref_nerf.preprocess_torch(pts, **o64.prep) + 1) / 2
            pts = torch.cat([pts[..., :2], pts[..., 2:] / o64.alt], -1).float().reshape(-1, 3)
            xg = p._last_hash_bwd[0].cpu()
            row["coords"] = {"differ_frac": float((xg != pts).any(1).double().mean()),
                             "max_abs": float((xg - pts).abs().max())}
            if "enc" in captured and getattr(p, "_last_d_enc", None) is not None:
                de_o = captured["enc"].grad.double()
                de_g = p._last_d_enc.double().cpu()
                row["d_enc"] = {"rows_differ_frac": float((de_o != de_g).any(1).double().mean()),
                                "elems_differ_frac": float((de_o != de_g).double().mean()),
                                "zero_flips": int(((de_o == 0) != (de_g == 0)).sum()),
                                "rel_l2": float((de_o - de_g).norm() / de_o.norm())}
                if "enc32" in captured:
                    de_3 = captured["enc32"].grad.double()
                    row["d_enc_f32arm"] = {
                        "rows_differ_frac": float((de_o != de_3).any(1).double().mean()),
                        "rel_l2": float((de_o - de_3).norm() / de_o.norm())}
                ds_g, dc_g = (t_.double().cpu() for t_ in p._last_field_grads)
                po_g = captured["pos_out"].grad.double()
                pos_out = captured["pos_out"].detach().double()
                ds_o = torch.where(pos_out[:, 0] > 0, po_g[:, 0], torch.zeros_like(po_g[:, 0]))
                live = pos_out[:, 0] > 0
                ds_gm = torch.where(live, ds_g.reshape(-1), torch.zeros_like(ds_o))
                rel = (ds_o - ds_gm).abs() / ds_o.abs().clamp_min(1e-30)
                top = torch.topk(torch.where(ds_o != 0, rel, torch.zeros_like(rel)), 6).indices
                row["d_sigma"] = {"gpu_vs_oracle_live": compare(ds_gm, ds_o),
                                  "differ_frac_live": float((ds_o != ds_gm)[live].double().mean()),
                                  "top": [(int(i), int(i) % a.samples, float(ds_o[i]),
                                           float(ds_gm[i]), float(pos_out[i, 0]))
                                          for i in top.tolist()]}
                dc_o = captured["dir_out"].grad.double()[:, :dc_g.shape[-1]]
                row["d_color"] = {"gpu_vs_oracle": compare(dc_g.reshape(dc_o.shape), dc_o)}
                rd = (de_o - de_g).abs().amax(1)
                top = torch.topk(rd, 4).indices.tolist()
                row["d_enc_top_rows"] = [{"row": r_, "sample": r_ % a.samples,
                                          "f64": de_o[r_].tolist(), "gpu": de_g[r_].tolist()}
                                         for r_ in top]
                # the oracle's f64 hash backward fed with the GPU's dL/denc, quantised as
                # tcnn's f16 gradient: isolates the GPU hash backward's accumulation
                x = p._last_hash_bwd[0].double().cpu().numpy()
                n_ent = int(g64.numel()) // 2
                cfg_g = (3, 16, 16, 1.3819, int(cfg["instant_ngp"]["encoding"]["log2_hashmap_size"]))
                gx = torch.from_numpy(ref_tcnn.hashgrid_bwd(x, (de_g * 128).numpy(), cfg_g, n_ent))
                gx = (gx.half() / 128).double()
                row["table_from_gpu_denc"] = {"vs_gpu": compare(g_gpu, gx), "vs_f64": compare(gx, g64)}
            rows.append(row)
            print(json.dumps(row), flush=True)
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "w") as f:
                json.dump(rows, f, indent=1)
        opt.step()


if __name__ == "__main__":
    main()
