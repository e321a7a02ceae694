"""Per-level anatomy of the hash-grid forward at bench size (VERDICT r02 "calibrate, then
cut, hash-forward traffic"): the bench scene's coordinates (90-view 512^2 synthetic
HARP2 scene -> fused sampler, 8,192 rays x 1,024 samples), the full 16-level grid and,
for every level l, a ONE-level grid with exactly level l's table size, resolution and
scale (its own table, offset 0), and every consecutive level pair (2p, 2p+1) likewise,
run through the same anr_hashgrid_fwd entry point.

Under rocprofv3 --pmc (tools/archive/r3_hash_level_pmc.sh) the hashgrid_fwd dispatches come in
the order printed as "launch_order", so each PMC row maps to (level | full, rep). The
one-level runs show what each level costs when it has the L2 to itself; the sum over
levels against the full run is the cross-level interference.

    python tools/hash_level_probe.py [--reps 3] [--out gpurun_out/hash_levels.json]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from atmonr_amd import _lib  # noqa: E402


def sub_grid(full, levels):
    """A grid of the given consecutive levels of ``full`` (their own table, offset 0)."""
    d = _lib.HashGridDesc()
    ctypes.memmove(ctypes.byref(d), ctypes.byref(full), ctypes.sizeof(d))
    d.n_levels = len(levels)
    base = full.offsets[levels[0]]
    for i, lv in enumerate(levels):
        d.offsets[i] = full.offsets[lv] - base
        d.resolutions[i] = full.resolutions[lv]
        d.scales[i] = full.scales[lv]
    d.offsets[len(levels)] = full.offsets[levels[-1] + 1] - base
    d.n_params = d.offsets[len(levels)] * full.n_features
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--views", type=int, default=90)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    from atmonr_amd.batch_loader import BatchLoader
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from atmonr_amd.samplers import sample_and_preprocess

    B, N = a.rays, a.samples
    M = B * N
    ds = SyntheticHARP2Dataset(n_views=a.views, img_size=a.img, device=dev, seed=0)
    batch = next(iter(BatchLoader(ds, B, shuffle=True, seed=0)))
    prep = ds.get_point_preprocessor("horizontal").params(ngp_remap=True, alt_compress=8.0)
    _, _, coords = sample_and_preprocess(batch, N, prep)
    x = coords.reshape(M, 3).contiguous()
    full = _lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19)
    table = ((torch.rand(full.n_params, device=dev) * 2 - 1) * 1e-2).half()
    s = _lib.stream(dev)

    levels = []
    for lv in range(full.n_levels):
        cell = torch.floor(x * full.scales[lv] + 0.5).to(torch.int64).view(B, N, 3)
        new = (cell[:, 1:] != cell[:, :-1]).any(-1).float().mean().item()
        size = full.offsets[lv + 1] - full.offsets[lv]
        res = full.resolutions[lv]
        levels.append({"level": lv, "res": res, "entries": size,
                       "hashed": res ** 3 > size, "table_kib_f16": size * 4 / 1024,
                       "new_cell_fraction": round(new, 4)})

    order = [["warmup", 0]]
    enc = torch.empty(M, 32, device=dev, dtype=torch.float16)
    _lib.call("anr_hashgrid_fwd", ctypes.byref(full), x.data_ptr(), 3, M, table.data_ptr(),
              _lib.F16, enc.data_ptr(), _lib.F16, 32, s)
    timer = _lib.KernelTimer()
    with timer:
        for r in range(a.reps):
            _lib.call("anr_hashgrid_fwd", ctypes.byref(full), x.data_ptr(), 3, M,
                      table.data_ptr(), _lib.F16, enc.data_ptr(), _lib.F16, 32, s, tag="full")
            order.append(["full", r])
        del enc
        groups = [[lv] for lv in range(full.n_levels)]
        groups += [[2 * p, 2 * p + 1] for p in range(full.n_levels // 2)]
        for g in groups:
            d = sub_grid(full, g)
            t1 = table[2 * full.offsets[g[0]]: 2 * full.offsets[g[-1] + 1]].contiguous()
            e1 = torch.empty(M, 2 * len(g), device=dev, dtype=torch.float16)
            tag = "level" + "_".join(map(str, g))
            for r in range(a.reps):
                _lib.call("anr_hashgrid_fwd", ctypes.byref(d), x.data_ptr(), 3, M,
                          t1.data_ptr(), _lib.F16, e1.data_ptr(), _lib.F16, 2 * len(g), s,
                          tag=tag)
                order.append([tag, r])
            del t1, e1
    summ = timer.summary()
    for row in levels:
        row["ms"] = round(summ[f"level{row['level']}"]["avg_ms"], 4)
        print(json.dumps(row), flush=True)
    pairs = {k: round(v["avg_ms"], 4) for k, v in summ.items() if k.count("_") == 1}
    rec = {"samples": M, "pair_ms": pairs, "full_ms": round(summ["full"]["avg_ms"], 4),
           "sum_level_ms": round(sum(r["ms"] for r in levels), 4),
           "levels": levels, "launch_order": order,
           "note": "one-level grids: level l's table alone; launches after the first "
                   "of each group run with a warm L2"}
    print(json.dumps({k: v for k, v in rec.items() if k not in ("levels", "launch_order")}))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(rec, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
