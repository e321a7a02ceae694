"""Standalone driver for the hash-grid kernels at bench size (profiling aid).

    python tools/hash_probe.py [--rays 8192] [--samples 1024] [--log2t 19] [--iters 3]

Ray-coherent coordinates (straight rays through the unit cube, samples in ray order, as
the sampler emits them), f16 table, f32 dL/denc. Prints HIP-event averages per kernel.
"""

from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--log2t", type=int, default=19)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--stats", action="store_true",
                    help="print per-level fraction of samples that enter a new cell")
    ap.add_argument("--synthetic-rays", action="store_true",
                    help="straight random rays instead of the bench scene's sampler output")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, N = args.rays, args.samples
    M = B * N
    if args.synthetic_rays:
        o = torch.rand(B, 1, 3, device=dev)
        d = torch.nn.functional.normalize(torch.randn(B, 1, 3, device=dev), dim=-1)
        t = torch.linspace(0, 1, N, device=dev).view(1, N, 1)
        x = ((o + 0.6 * d * t) % 1.0).reshape(M, 3).contiguous()
    else:  # the bench workload's coordinates: synthetic HARP2 scene -> fused sampler
        sys.path.insert(0, ROOT)
        from atmonr_amd.batch_loader import BatchLoader
        from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
        from atmonr_amd.samplers import sample_and_preprocess

        ds = SyntheticHARP2Dataset(n_views=8, img_size=512, device=dev, seed=0)
        batch = next(iter(BatchLoader(ds, B, shuffle=True, seed=0)))
        prep = ds.get_point_preprocessor("horizontal").params(ngp_remap=True, alt_compress=8.0)
        _, _, coords = sample_and_preprocess(batch, N, prep)
        x = coords.reshape(M, 3).contiguous()
    desc = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, args.log2t)
    table = ((torch.rand(desc.n_params, device=dev) * 2 - 1) * 1e-2).half()
    enc = torch.empty(M, 32, device=dev, dtype=torch.float16)
    denc = torch.randn(M, 32, device=dev) * 1e-3
    grad = torch.zeros(desc.n_params, device=dev)
    if args.stats:
        tot = 0.0
        for lv in range(desc.n_levels):
            cell = torch.floor(x * desc.scales[lv] + 0.5).to(torch.int64).view(B, N, 3)
            ch = (cell[:, 1:] != cell[:, :-1]).any(-1).float().mean().item()
            tot += ch
            print(f"level {lv:2d} res {desc.resolutions[lv]:5d} new-cell fraction {ch:.3f}")
        print(f"mean cells entered per sample over levels: {tot:.2f} (of {desc.n_levels})")
    s = _lib.stream(dev)
    timer = _lib.KernelTimer()
    with timer:
        for _ in range(args.iters):
            _lib.call("anr_hashgrid_fwd", ctypes.byref(desc), x.data_ptr(), 3, M,
                      table.data_ptr(), _lib.F16, enc.data_ptr(), _lib.F16, 32, s,
                      tag="hash_fwd")
            _lib.call("anr_hashgrid_bwd", ctypes.byref(desc), x.data_ptr(), 3, M,
                      denc.data_ptr(), _lib.F32, 32, grad.data_ptr(), s, tag="hash_bwd")
    torch.cuda.synchronize()
    for k, v in timer.summary().items():
        print(f"{k:10s} avg {v['avg_ms']:.4f} ms  ({v['launches']} calls)")


if __name__ == "__main__":
    main()
