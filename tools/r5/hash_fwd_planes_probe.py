"""Hash-grid forward v6 (rows) vs v9 (level-quad planes, one lane per sample) on the
bench's coordinates (profiling aid, r05).

    python tools/r5/hash_fwd_planes_probe.py [--iters 20]
"""

from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "atmospheric-neural-rendering_amd")]

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402


def timed(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for it in range(iters + 2):
        torch.cuda.synchronize()
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        if it >= 2:
            ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.samplers import sample_and_preprocess

    ds = SyntheticHARP2Dataset(n_views=90, img_size=512, device=dev, seed=0)
    batch = next(iter(BatchLoader(ds, a.rays, shuffle=True, seed=0)))
    prep = ds.get_point_preprocessor("horizontal").params(ngp_remap=True, alt_compress=8.0)
    _, _, coords = sample_and_preprocess(batch, a.samples, prep)
    x = coords.reshape(-1, 3).contiguous()
    M = x.shape[0]
    desc = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    g = torch.Generator(device=dev).manual_seed(0)
    table = ((torch.rand(desc.n_params, device=dev, generator=g) * 2 - 1) * 1e-2).half()
    rows = torch.empty(M, 32, device=dev, dtype=torch.float16)
    planes = torch.empty(4, M, 8, device=dev, dtype=torch.float16)
    s = _lib.stream(dev)

    def f_rows():
        _lib.call("anr_hashgrid_fwd", ctypes.byref(desc), x.data_ptr(), 3, M, table.data_ptr(),
                  _lib.F16, rows.data_ptr(), _lib.F16, 32, s)

    def f_planes():
        _lib.call("anr_hashgrid_fwd_planes", ctypes.byref(desc), x.data_ptr(), 3, M,
                  table.data_ptr(), _lib.F16, planes.data_ptr(), 8 * M, s)

    t_r = timed(f_rows, a.iters)
    t_p = timed(f_planes, a.iters)
    same = torch.equal(rows.view(M, 4, 8).permute(1, 0, 2), planes)
    print(f"M={M} rows(v6) median {t_r[0]:.4f} "
          f"min {t_r[1]:.4f} ms | planes(v9) median {t_p[0]:.4f} min {t_p[1]:.4f} ms | "
          f"bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
