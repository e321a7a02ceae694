"""Diagnostic: one test_ingp_field_matches_oracle case run through every field backward
generation (anr_ingp_field_force_bwd modes 0-2), twice each, with the error of every
gradient segment against the f64 oracle and between modes.

usage: python tools/field_case_diag.py [width nhd R mma]   (GPU)
"""

import ctypes
import sys

import torch

sys.path.insert(0, ".")
import tests.conftest  # noqa: E402,F401  (puts the package and oracle on sys.path)

from atmonr_amd import _lib  # noqa: E402
from tests.test_kernels_gpu import _field_preacts, _field_ref  # noqa: E402


def main():
    width, nhd, R = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 2, 29)
    mma = sys.argv[4] if len(sys.argv) > 4 else "f16"
    dev = torch.device("cuda", 0)
    half = "bf16" if mma == "bf16" else True
    code = _lib.BF16 if mma == "bf16" else _lib.F16
    nb, n_per_ray = 4, 37
    M = n_per_ray * R
    gen = torch.Generator().manual_seed(1000 * width + 10 * nhd + R)
    pdsc = _lib.mlp_desc(32, 16, width, 1, False)
    ddsc = _lib.mlp_desc(19, nb, width, nhd, False)
    lib = _lib.load()
    n_pp = lib.anr_mlp_n_params(ctypes.byref(pdsc))
    n_pd = lib.anr_mlp_n_params(ctypes.byref(ddsc))
    pp = torch.randn(n_pp, generator=gen) * (2.0 / 32) ** 0.5
    pd = torch.randn(n_pd, generator=gen) * (2.0 / width) ** 0.5
    enc = torch.rand(M, 32, generator=gen) * 2 - 1
    dirs = torch.nn.functional.normalize(torch.randn(R, 3, generator=gen), dim=1)
    for _ in range(40):
        tied = _field_preacts(enc, dirs, n_per_ray, pp, pd, width, nhd, half) < 2e-3
        if not tied.any():
            break
        enc[tied] = torch.rand(int(tied.sum()), 32, generator=gen) * 2 - 1
    enc_h = enc.half()
    s = _lib.stream(dev)
    pp_d, pd_d, enc_d, dirs_d = pp.to(dev), pd.to(dev), enc_h.to(dev), dirs.to(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(ctypes.byref(pdsc), ctypes.byref(ddsc)),
                         device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", ctypes.byref(pdsc), ctypes.byref(ddsc), code,
              pp_d.data_ptr(), pd_d.data_ptr(), packed.data_ptr(), s)
    e64 = enc_h.double().requires_grad_(True)
    pr_p = pp.double().requires_grad_(True)
    pr_d = pd.double().requires_grad_(True)
    rs, rc, _, _ = _field_ref(e64, dirs, n_per_ray, pr_p, pr_d, width, nhd, nb, half)
    dcol = torch.randn(M, nb, generator=gen) * 1e-2
    dsig = torch.randn(M, generator=gen) * 1e-3
    ((rc * dcol.double()).sum() + (rs * dsig.double()).sum()).backward()
    dcol_d, dsig_d = dcol.to(dev), dsig.to(dev)
    ws_bytes = lib.anr_ingp_field_bwd_workspace_bytes(ctypes.byref(pdsc), ctypes.byref(ddsc),
                                                      code, M)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev)
    segs = {"D0": (0, width * 32)}
    off = width * 32
    for k in range(1, nhd):
        segs[f"D{k}"] = (off, off + width * width)
        off += width * width
    segs[f"D{nhd}"] = (off, n_pd)
    ref_d = pr_d.grad
    scale = ref_d.abs().max().item()
    outs = {}
    for mode in (0, 1, 2):
        for rep in range(2):
            prev = lib.anr_ingp_field_force_bwd(mode)
            d_enc = torch.zeros(M, 32, device=dev)
            g_pos = torch.zeros(n_pp, device=dev)
            g_dir = torch.zeros(n_pd, device=dev)
            _lib.call("anr_ingp_field_bwd", ctypes.byref(pdsc), ctypes.byref(ddsc), code,
                      packed.data_ptr(), enc_d.data_ptr(), 32, dirs_d.data_ptr(), n_per_ray, M,
                      dsig_d.data_ptr(), dcol_d.data_ptr(), nb, d_enc.data_ptr(), 32,
                      g_pos.data_ptr(), g_dir.data_ptr(), ws.data_ptr() if ws_bytes else None,
                      ws_bytes, s)
            torch.cuda.synchronize()
            lib.anr_ingp_field_force_bwd(prev)
            gd = g_dir.double().cpu()
            err = {k: (gd[a:b] - ref_d[a:b]).abs().max().item() / scale for k, (a, b) in segs.items()}
            i = int((gd - ref_d).abs().argmax())
            print(f"mode {mode} rep {rep}: g_dir rel-max err by segment "
                  + " ".join(f"{k}={v:.3e}" for k, v in err.items())
                  + f" | argmax {i} got {gd[i]:.6f} ref {ref_d[i]:.6f}"
                  + f" | d_enc {(d_enc.double().cpu() - e64.grad).abs().max().item() / e64.grad.abs().max().item():.3e}"
                  + f" g_pos {(g_pos.double().cpu() - pr_p.grad).abs().max().item() / pr_p.grad.abs().max().item():.3e}",
                  flush=True)
            outs[(mode, rep)] = (d_enc.cpu(), g_pos.cpu(), gd)
    # determinism: 40 more launches per mode, each compared with the first
    for mode in (0, 1, 2):
        prev = lib.anr_ingp_field_force_bwd(mode)
        worst, bad = 0.0, 0
        for rep in range(40):
            d_enc = torch.zeros(M, 32, device=dev)
            g_pos = torch.zeros(n_pp, device=dev)
            g_dir = torch.zeros(n_pd, device=dev)
            _lib.call("anr_ingp_field_bwd", ctypes.byref(pdsc), ctypes.byref(ddsc), code,
                      packed.data_ptr(), enc_d.data_ptr(), 32, dirs_d.data_ptr(), n_per_ray, M,
                      dsig_d.data_ptr(), dcol_d.data_ptr(), nb, d_enc.data_ptr(), 32,
                      g_pos.data_ptr(), g_dir.data_ptr(), ws.data_ptr() if ws_bytes else None,
                      ws_bytes, s)
            torch.cuda.synchronize()
            dd = (g_dir.double().cpu() - outs[(mode, 0)][2]).abs().max().item() / scale
            de = int((d_enc.cpu() != outs[(mode, 0)][0]).sum())
            worst = max(worst, dd)
            bad += int(dd > 1e-5 or de > 0)
        lib.anr_ingp_field_force_bwd(prev)
        print(f"mode {mode}: 40 relaunches, worst g_dir rel diff {worst:.3e}, "
              f"launches off by > 1e-5 or any d_enc bit: {bad}", flush=True)
    for m in (0, 2):
        a, b = outs[(m, 0)], outs[(1, 0)]
        print(f"mode {m} vs 1: d_enc equal {torch.equal(a[0], b[0])}, g_dir max diff "
              f"{(a[2] - b[2]).abs().max().item():.3e}")
    print("rep-to-rep g_dir max diff (mode 1):",
          (outs[(1, 0)][2] - outs[(1, 1)][2]).abs().max().item())


if __name__ == "__main__":
    main()
