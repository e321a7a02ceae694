"""Diagnostic: field backward generation 0 (LDS tiles) vs 1 (register-transposed) on the
same inputs; prints per-weight-block relative differences and d_enc mismatch counts."""
import ctypes
import sys

import torch

sys.path.insert(0, "atmospheric-neural-rendering_amd")
from atmonr_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
for mma in ("f16", "bf16"):
    for width, nhd in ((64, 2), (32, 1)):
        nb, R, npr = 4, 29, 37
        M = R * npr
        code = _lib.BF16 if mma == "bf16" else _lib.F16
        g = torch.Generator(device=dev).manual_seed(3)
        pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
        pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
        pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
        pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
        enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
        dirs = torch.rand(R, 3, device=dev, generator=g)
        s = _lib.stream(dev)
        packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
        _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(), packed.data_ptr(), s)
        dcol = torch.randn(M, nb, device=dev, generator=g) * 1e-2
        dsig = torch.randn(M, device=dev, generator=g) * 1e-3
        wsb = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, code, M)
        ws = torch.empty(max(1, wsb // 4), device=dev)
        out = {}
        for mode in (0, 1):
            lib.anr_ingp_field_force_bwd(mode)
            d_enc = torch.zeros(M, 32, device=dev)
            gp, gd = torch.zeros_like(pp), torch.zeros_like(pd)
            _lib.call("anr_ingp_field_bwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
                      dirs.data_ptr(), npr, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                      d_enc.data_ptr(), 32, gp.data_ptr(), gd.data_ptr(),
                      ws.data_ptr() if wsb else None, wsb, s)
            torch.cuda.synchronize()
            out[mode] = (d_enc.cpu(), gp.cpu(), gd.cpu())
        lib.anr_ingp_field_force_bwd(1)
        W = width
        pblk = {"P0": (0, 32 * W), "P1": (32 * W, 48 * W)}
        dblk = {"D0": (0, 32 * W)}
        if nhd == 2:
            dblk["D1"] = (32 * W, 32 * W + W * W)
        off = 32 * W + (nhd - 1) * W * W
        dblk["D2"] = (off, off + 16 * W)
        line = [f"{mma} W={W} nhd={nhd}: d_enc mismatches {(out[0][0] != out[1][0]).sum().item()}"
                f" maxdiff {(out[0][0] - out[1][0]).abs().max().item():.3e}"]
        for name, (a, b) in pblk.items():
            x, y = out[1][1][a:b], out[0][1][a:b]
            line.append(f"{name} {((x - y).norm() / y.norm()).item():.2e}")
        for name, (a, b) in dblk.items():
            x, y = out[1][2][a:b], out[0][2][a:b]
            e = (x - y).abs().view(-1, 32 if name == 'D0' else W)
            line.append(f"{name} {((x - y).norm() / y.norm()).item():.2e} worst(row,col)="
                        f"{divmod(int(e.argmax()), e.shape[1])}")
        print("  ".join(line), flush=True)
