"""Field backward alone at the bench shape (8,192 rays x 1,024 samples, W=64, 2 dir hidden
layers, f16), for PMC passes and timing (the r03 A/B generations were removed in r04).
Random weights, encodings and output gradients; prints the mean launch time over --iters
launches (HIP events on the launch stream).

usage: python tools/field_bwd_pmc.py [--iters 20] [--rays 8192]
"""

import argparse
import ctypes
import json
import sys

import torch

sys.path.insert(0, "atmospheric-neural-rendering_amd")
from atmonr_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--spr", type=int, default=1024)
    ap.add_argument("--mma", default="f16", choices=["f16", "bf16"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    width, nhd, nb = 64, 2, 4
    R, npr = args.rays, args.spr
    M = R * npr
    code = _lib.BF16 if args.mma == "bf16" else _lib.F16
    g = torch.Generator(device=dev).manual_seed(5)
    pdsc, ddsc = _lib.mlp_desc(32, 16, width, 1, False), _lib.mlp_desc(19, nb, width, nhd, False)
    pb, db = ctypes.byref(pdsc), ctypes.byref(ddsc)
    pp = torch.randn(lib.anr_mlp_n_params(pb), device=dev, generator=g) * (2.0 / 32) ** 0.5
    pd = torch.randn(lib.anr_mlp_n_params(db), device=dev, generator=g) * (2.0 / width) ** 0.5
    enc = (torch.rand(M, 32, device=dev, generator=g) * 2 - 1).half()
    dirs = torch.rand(R, 3, device=dev, generator=g)
    s = _lib.stream(dev)
    packed = torch.empty(lib.anr_ingp_field_packed_size(pb, db), device=dev, dtype=torch.float16)
    _lib.call("anr_ingp_field_pack", pb, db, code, pp.data_ptr(), pd.data_ptr(),
              packed.data_ptr(), s)
    dcol = torch.randn(M, nb, device=dev, generator=g) * 1e-3
    dsig = torch.randn(M, device=dev, generator=g) * 1e-3
    wsb = lib.anr_ingp_field_bwd_workspace_bytes(pb, db, code, M)
    ws = torch.empty(max(1, wsb // 4), device=dev)
    d_enc = torch.empty(M, 32, device=dev)
    gp, gd = torch.zeros_like(pp), torch.zeros_like(pd)

    def launch():
        _lib.call("anr_ingp_field_bwd", pb, db, code, packed.data_ptr(), enc.data_ptr(), 32,
                  dirs.data_ptr(), npr, M, dsig.data_ptr(), dcol.data_ptr(), nb,
                  d_enc.data_ptr(), 32, gp.data_ptr(), gd.data_ptr(),
                  ws.data_ptr() if wsb else None, wsb, s)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    # _lib.stream() is torch's current stream, which the events record on
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"mma": args.mma, "M": M,
                      "ms_per_launch": e0.elapsed_time(e1) / args.iters}))


if __name__ == "__main__":
    main()
