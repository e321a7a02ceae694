"""A/B of the hash-grid backward generations at bench size (profiling aid).

    python tools/hash_bwd_ab.py [--modes 0,1] [--iters 10]

Bench coordinates (synthetic HARP2 scene -> fused sampler, 8192 rays x 1024 samples), f32
dL/denc, f32 gradient table. Prints the HIP-event average per mode and the relative L2
difference of each mode's gradient from the first mode's. (The r02 log's mode 8, the
segment-flush backward v3, was removed from the library after measuring it.)
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="0,1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, N = args.rays, args.samples
    M = B * N
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.samplers import sample_and_preprocess

    ds = SyntheticHARP2Dataset(n_views=8, img_size=512, device=dev, seed=0)
    batch = next(iter(BatchLoader(ds, B, shuffle=True, seed=0)))
    prep = ds.get_point_preprocessor("horizontal").params(ngp_remap=True, alt_compress=8.0)
    _, _, coords = sample_and_preprocess(batch, N, prep)
    x = coords.reshape(M, 3).contiguous()
    desc = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    denc = torch.randn(M, 32, device=dev) * 1e-3
    lib = _lib.load()
    s = _lib.stream(dev)
    grads = {}
    for mode in [int(m) for m in args.modes.split(",")]:
        grad = torch.zeros(desc.n_params, device=dev)
        prev = lib.anr_hashgrid_force_v1(mode)
        timer = _lib.KernelTimer()
        for it in range(args.iters + 2):
            if it == 2:
                timer.__enter__()
            if it == args.iters + 1:
                grad.zero_()
            _lib.call("anr_hashgrid_bwd", ctypes.byref(desc), x.data_ptr(), 3, M,
                      denc.data_ptr(), _lib.F32, 32, grad.data_ptr(), s,
                      tag=f"hash_bwd_m{mode}")
        timer.__exit__(None, None, None)
        torch.cuda.synchronize()
        lib.anr_hashgrid_force_v1(prev)
        for k, v in timer.summary().items():
            print(f"mode {mode}: {k} avg {v['avg_ms']:.4f} ms ({v['launches']} calls)", flush=True)
        grads[mode] = grad
    first = next(iter(grads.values()))
    for m, g in grads.items():
        rel = ((g - first).norm() / first.norm().clamp_min(1e-30)).item()
        print(f"mode {m}: rel L2 vs first {rel:.3e}", flush=True)


if __name__ == "__main__":
    main()
