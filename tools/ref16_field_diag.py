"""Where the GPU's f16 hash-table gradient departs from the oracle's (GPU diagnostic).

One Instant-NGP step (8-view 16x16 scene, 200 rays x 64 samples) in reference numerics
on the GPU and in reference semantics in the oracle, same parameters / rays / draws;
compares dL/dpos_enc sample by sample and the hash-table gradient level by level.

    python tools/ref16_field_diag.py [--numerics reference|build]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--numerics", default="reference")
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--rays", type=int, default=200)
    ap.add_argument("--psnr-batch", action="store_true",
                    help="the first batch and draws of tests/ingp_psnr.py instead")
    a = ap.parse_args()
    import __graft_entry__ as ge
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.pipelines.instant_ngp import InstantNGPPipeline
    from oracle import ref_ingp, ref_tcnn

    dev = torch.device("cuda:0")
    torch.set_num_threads(16)
    scene = SyntheticHARP2Dataset(n_views=8, img_size=16, device=dev, seed=0)
    cfg = ge._ingp_config(a.samples)
    p = InstantNGPPipeline(cfg, scene, fused=True, seed=5, numerics=a.numerics)
    p.send_tensors_to(dev)
    p._keep_d_enc = True
    pp = scene.get_point_preprocessor("horizontal")
    o = ref_ingp.RefInstantNGP(cfg, p.state_dict(), ref_ingp.prep_kwargs(pp), p.scale,
                               scene.max_i, half=True,
                               semantics="reference" if a.numerics == "reference" else "build")
    B, N = a.rays, a.samples
    if a.psnr_batch:
        from tests import ingp_psnr
        batch = next(iter(BatchLoader(scene, B, seed=ingp_psnr.SEED_BATCH)))
        u = torch.rand(B, N, generator=torch.Generator().manual_seed(ingp_psnr.SEED_U))
    else:
        batch = next(iter(BatchLoader(scene, B, seed=1)))
        u = torch.rand(B, N, generator=torch.Generator().manual_seed(2))
    p.compute_loss(batch, p.forward(batch, u=u.to(dev))).backward()
    torch.cuda.synchronize()
    # oracle, with dL/dpos_enc retained
    cb = ref_ingp.cpu_batch(batch)
    captured = {}
    orig = ref_ingp._TcnnCall.apply

    def spy(x, params, fn, *rest):
        y = orig(x, params, fn, *rest)
        if params is o.params["pos_encoder"]:
            y.retain_grad()
            captured["enc"] = y
        return y
    ref_ingp._TcnnCall.apply = spy
    res = o.forward(cb, u)
    o.loss(cb, res).backward()
    ref_ingp._TcnnCall.apply = orig
    out = {}
    if "enc" in captured:
        ge_ = p._last_d_enc.double().cpu()
        go = captured["enc"].grad.double()
        out["d_enc_equal_frac"] = (ge_ == go).double().mean().item()
        out["d_enc_rel_l2"] = ((ge_ - go).norm() / go.norm()).item()
        d = (ge_ - go).abs()
        out["d_enc_max_abs_diff"] = d.max().item()
        out["d_enc_max_abs"] = go.abs().max().item()
        out["d_enc_rel_l2_per_level"] = [
            ((ge_[:, 2 * l:2 * l + 2] - go[:, 2 * l:2 * l + 2]).norm()
             / go[:, 2 * l:2 * l + 2].norm().clamp_min(1e-300)).item() for l in range(16)]
    if "enc" in captured:
        # which samples differ, and how close their pos-MLP pre-activations are to 0
        rows = torch.nonzero((ge_ != go).any(1)).view(-1)
        out["rows_differing"] = int(rows.numel())
        enc = captured["enc"].detach().double()
        W0 = o.params["pos_mlp"].detach()[:64 * 32].half().double().view(64, 32)
        W1 = o.params["pos_mlp"].detach()[64 * 32:].half().double().view(16, 64)
        pre = enc @ W0.t()
        hid = torch.relu(pre).half().double()
        po = hid @ W1.t()
        absmin = pre.abs().min(1).values
        out["rows_differing_sample_pos"] = (rows % N).tolist()[:64]
        out["rows_differing_min_abs_preact"] = absmin[rows].tolist()[:32]
        out["all_rows_min_abs_preact_median"] = absmin.median().item()
        out["rows_differing_pos_out0"] = po[rows, 0].tolist()[:32]
        rel = ((ge_ - go).abs().max(1).values / go.abs().max(1).values.clamp_min(1e-30))[rows]
        out["rows_differing_rel_maxdiff"] = rel.tolist()[:32]
        out["rows_differing_d_enc_gpu_norm"] = ge_[rows].norm(dim=1).tolist()[:16]
        out["rows_differing_d_enc_oracle_norm"] = go[rows].norm(dim=1).tolist()[:16]
    # table gradient level by level
    offs, sizes, res_, scales, _ = ref_tcnn.grid_levels(3, 16, 16, 1.3819, 19)
    gg = p.pos_encoder.params.grad.double().cpu()
    go = o.params["pos_encoder"].grad
    per = []
    for l in range(16):
        s, e = 2 * offs[l], 2 * (offs[l] + sizes[l])
        per.append(((gg[s:e] - go[s:e]).norm() / go[s:e].norm().clamp_min(1e-300)).item())
    out["table_rel_l2_per_level"] = per
    out["table_norm_per_level"] = [go[2 * offs[l]:2 * (offs[l] + sizes[l])].norm().item()
                                   for l in range(16)]
    out["table_rel_l2"] = ((gg - go).norm() / go.norm()).item()
    for m in ("pos_mlp", "dir_mlp", "surf_encoder", "surf_mlp"):
        g1 = getattr(p, m).params.grad.double().cpu()
        g2 = o.params[m].grad
        out[m] = ((g1 - g2).norm() / g2.norm()).item()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
