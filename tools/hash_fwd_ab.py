"""A/B of the hash-grid forward generations at bench size (profiling aid).

    python tools/hash_fwd_ab.py [--modes 1,0] [--iters 10] [--log2t 19]

Bench coordinates (synthetic HARP2 scene -> fused sampler, 8192 rays x 1024 samples), f16
table, f16 output; modes as anr_hashgrid_force_v1 (0 = v6, 1 = v1), or "p" for
anr_hashgrid_fwd_planar (v8, level-pair planes, converted back to rows for the check;
removed from the library after profiles/r03_hash_levels.md §3).
Every mode's output is compared bit for bit with mode 1's (or mode 0's). Prints the HIP-event average per mode. (The r02 log's
mode 7, a level-major-plane experiment, was removed from the library after measuring it.)
"""

from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--log2t", type=int, default=19)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="1,0")
    ap.add_argument("--views", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, N = args.rays, args.samples
    M = B * N
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.samplers import sample_and_preprocess

    ds = SyntheticHARP2Dataset(n_views=args.views, img_size=512, device=dev, seed=0)
    batch = next(iter(BatchLoader(ds, B, shuffle=True, seed=0)))
    prep = ds.get_point_preprocessor("horizontal").params(ngp_remap=True, alt_compress=8.0)
    _, _, coords = sample_and_preprocess(batch, N, prep)
    x = coords.reshape(M, 3).contiguous()
    desc = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, args.log2t)
    table = ((torch.rand(desc.n_params, device=dev) * 2 - 1) * 1e-2).half()
    lib = _lib.load()
    s = _lib.stream(dev)
    outs = {}
    for mode in [m if m == "p" else int(m) for m in args.modes.split(",")]:
        enc = torch.empty(M, 32, device=dev, dtype=torch.float16)
        planes = torch.empty(8, M, 4, device=dev, dtype=torch.float16)
        prev = lib.anr_hashgrid_force_v1(0 if mode == "p" else mode)
        timer = _lib.KernelTimer()
        for it in range(args.iters + 2):
            if it == 2:
                timer.__enter__()
            if mode == "p":
                _lib.call("anr_hashgrid_fwd_planar", ctypes.byref(desc), x.data_ptr(), 3, M,
                          table.data_ptr(), _lib.F16, planes.data_ptr(), _lib.F16, s,
                          tag="hash_fwd_planar")
            else:
                _lib.call("anr_hashgrid_fwd", ctypes.byref(desc), x.data_ptr(), 3, M,
                          table.data_ptr(), _lib.F16, enc.data_ptr(), _lib.F16, 32, s,
                          tag=f"hash_fwd_m{mode}")
        timer.__exit__(None, None, None)
        torch.cuda.synchronize()
        lib.anr_hashgrid_force_v1(prev)
        for k, v in timer.summary().items():
            print(f"mode {mode}: {k} avg {v['avg_ms']:.4f} ms ({v['launches']} calls)", flush=True)
        if mode == "p":
            enc = planes.permute(1, 0, 2).reshape(M, 32)
        outs[mode] = enc
    ref = outs.get(1, outs.get(0))
    if ref is not None:
        for m, o in outs.items():
            print(f"mode {m} equal to mode {1 if 1 in outs else 0}: {torch.equal(o, ref)}",
                  flush=True)


if __name__ == "__main__":
    main()
