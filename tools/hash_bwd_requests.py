"""Memory-side atomic requests of the hash-grid backward, by cause, simulated on the CPU.

VERDICT r03 "hash backward: attack the 25 % request fill; first count requests by cause".
The v2 backward (csrc/hashgrid.hip hashgrid_bwd_v2_kernel) gives each level 4 lanes
(x-offset b, feature f) that hold the f32 gradient of the NC = 4 (y, z) corners of the
current cell, and issues one no-return f32 atomic per held corner when it leaves: the
cell changes so that the corner is no longer one of the new cell's (x changed: all four;
y / z by one: two), and at the chunk end (all four). One wave instruction of 16 levels x
4 lanes goes to memory as one 64-B request per distinct 64-B segment it touches
(MI355X_MICROARCH.md "Global float atomics"): the 4 lanes of a level touch entries
(x, x+1) x 2 features = 16 B, one segment unless the pair straddles a segment edge.

This replays that walk on the bench's sample coordinates (the 90-view 512^2 synthetic
scene, rays drawn at random, 1,024 stratified samples per ray, the oracle's sampler and
f64 preprocessor, f32 cell arithmetic as the kernel) and counts, per level:

  move_x      requests of corners flushed because the cell moved in x
  move_yz     ... moved in y / z only (the corners that leave)
  chunk_end   requests of the chunk-end flush
  -> requests per sample, and the same for other chunk lengths K and for the "segment
     hold" variant: accumulators held per 64-B segment (8 x-neighbours x 2 features),
     flushed as ONE request when no corner of the current cell lies in it any more.

Usage: python tools/hash_bwd_requests.py [--rays 512] [--views 90] [--img 512]
Output: JSON on stdout (profiles/r04_hash_bwd_requests.json).
"""

from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "atmospheric-neural-rendering_amd"))

PRIMES = (1, 2654435761, 805459861)


def levels(n_levels=16, base=16, pls=1.3819, log2t=19, D=3):
    """tcnn GridEncoding level geometry restated in numpy (scales within 1 f32 ulp of
    anr_hashgrid_init's; main() uses the library's own)."""
    out, off = [], 0
    l2 = np.float32(math.log2(pls))
    for lv in range(n_levels):
        scale = np.float32(np.exp2(np.float32(lv) * l2) * np.float32(base) - np.float32(1.0))
        res = int(math.ceil(float(scale))) + 1
        n = min(((res ** D + 7) // 8) * 8, 1 << log2t)
        out.append({"scale": scale, "res": res, "T": n, "offset": off, "hashed": res ** D > n})
        off += n
    return out


def corner_index(lv, g):
    """Entry index of lattice points g (..., 3) uint64 within the level (grid_index)."""
    T, res = lv["T"], lv["res"]
    if lv["hashed"]:
        h = np.zeros(g.shape[:-1], dtype=np.uint64)
        for d in range(3):
            h ^= (g[..., d] * np.uint64(PRIMES[d])) & np.uint64(0xFFFFFFFF)
        return h & np.uint64(T - 1)
    s = (g[..., 0] + g[..., 1] * np.uint64(res) + g[..., 2] * np.uint64(res * res))
    s = s & np.uint64(0xFFFFFFFF)
    return s % np.uint64(T)


def segs(lv, idx):
    """64-B segment of entry idx (8-B f32 gradient pairs, level table 64-B aligned)."""
    return (np.uint64(lv["offset"]) + idx) >> np.uint64(3)


def coords(n_rays, views, img, n_samples, seed=0):
    from atmonr_amd.datasets.synthetic import SyntheticHARP2Dataset
    from oracle import ref_nerf, ref_path

    ds = SyntheticHARP2Dataset(n_views=views, img_size=img, device="cpu", seed=0)
    pp = ds._prep
    gen = torch.Generator().manual_seed(seed)
    idx = torch.randint(0, len(ds), (n_rays,), generator=gen)
    b = ds.__getbatch__(idx)
    u = torch.rand(n_rays, n_samples, generator=gen)
    pts, _ = ref_path.sample_uniform_bins(b["origin"], b["dir"], b["len"], u=u,
                                          n_bins=n_samples)
    prep = dict(scale=pp.scale, offset=torch.tensor(pp.offset, dtype=torch.float64),
                lat_min=pp.lat_min, lat_range=pp.lat_range, lon_min=pp.lon_min,
                lon_range=pp.lon_range, h0=pp.ray_origin_height, shift_lon=pp.shift_lon)
    c = ref_nerf.preprocess_torch(pts.double(), **prep)
    c = (c + 1) / 2
    c[..., 2] = c[..., 2] / 8.0  # alt_compress_factor
    return c.float().numpy().reshape(-1, 3)


def fma_pos(lv, x):
    """fmaf(scale, x, 0.5) in f32: the f64 product of two f32 values is exact, so one
    rounding to f32 of product + 0.5 is the fused result."""
    return (np.float64(lv["scale"]) * x.astype(np.float64) + 0.5).astype(np.float32)


def walk(lv, x, K):
    """Per-cause request counts of the v2 walk over x (M, 3) f32 in chunks of K."""
    M = x.shape[0]
    pos = fma_pos(lv, x)
    cell = np.floor(pos).astype(np.int64)
    chunk = np.arange(M) // K
    new_chunk = np.r_[True, chunk[1:] != chunk[:-1]]
    moved = np.r_[False, np.any(cell[1:] != cell[:-1], axis=1)] & ~new_chunk
    t = np.nonzero(moved)[0]
    old, new = cell[t - 1], cell[t]
    keepx = old[:, 0] == new[:, 0]
    dl = old - new
    out = {"move_x": 0, "move_yz": 0, "chunk_end": 0, "cell_moves": int(t.size)}
    cb = [(cy, cz) for cz in (0, 1) for cy in (0, 1)]

    def pair_requests(c0, cy, cz):
        # segments of entries (x, y+cy, z+cz) and (x+1, ...), as the 4 lanes touch them
        g0 = np.stack([c0[:, 0], c0[:, 1] + cy, c0[:, 2] + cz], 1).astype(np.uint64)
        g1 = g0.copy()
        g1[:, 0] += np.uint64(1)
        s0, s1 = segs(lv, corner_index(lv, g0)), segs(lv, corner_index(lv, g1))
        return 1 + (s0 != s1).astype(np.int64)

    for cy, cz in cb:
        leaves = ~keepx | ((cy + dl[:, 1]) < 0) | ((cy + dl[:, 1]) > 1) | \
                 ((cz + dl[:, 2]) < 0) | ((cz + dl[:, 2]) > 1)
        r = pair_requests(old, cy, cz)
        out["move_x"] += int(r[leaves & ~keepx].sum())
        out["move_yz"] += int(r[leaves & keepx].sum())
    last = np.r_[np.nonzero(new_chunk)[0][1:] - 1, M - 1]
    for cy, cz in cb:
        out["chunk_end"] += int(pair_requests(cell[last], cy, cz).sum())
    return out


def walk_segment_hold(lv, x, K):
    """Requests if every 64-B segment were held until no corner of the current cell lies
    in it (one full request per release), chunk-end flush of the held segments."""
    M = x.shape[0]
    pos = fma_pos(lv, x)
    cell = np.floor(pos).astype(np.int64)
    corners = []
    for cz in (0, 1):
        for cy in (0, 1):
            for cx in (0, 1):
                g = np.stack([cell[:, 0] + cx, cell[:, 1] + cy, cell[:, 2] + cz], 1)
                corners.append(segs(lv, corner_index(lv, g.astype(np.uint64))))
    S = np.stack(corners, 1)  # (M, 8) segments of each sample's cell
    req = 0
    for k0 in range(0, M, K):
        held = set()
        for m in range(k0, min(M, k0 + K)):
            cur = set(S[m].tolist())
            req += len(held - cur)
            held = cur
        req += len(held)
    return req


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=512)
    ap.add_argument("--views", type=int, default=90)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--hold-rays", type=int, default=32,
                    help="rays for the (slow, pure-Python) segment-hold variant")
    a = ap.parse_args()
    x = coords(a.rays, a.views, a.img, a.samples)
    M = x.shape[0]
    from atmonr_amd import _lib
    from tools.hash_requests import level_geometry

    # the kernel's own level geometry (anr_hashgrid_init), as tools/hash_requests.py
    L = level_geometry(_lib.hashgrid_desc(3, 16, 2, 16, 1.3819, 19))
    res = {"rays": a.rays, "samples_per_ray": a.samples, "scene": f"{a.views}x{a.img}^2",
           "chunks": {}}
    for K in (32, 64, 128, 256, 512, 1024):
        per = []
        tot = {"move_x": 0, "move_yz": 0, "chunk_end": 0, "cell_moves": 0}
        for lv in L:
            w = walk(lv, x, K)
            per.append({k: round(v / M, 4) for k, v in w.items()})
            for k in tot:
                tot[k] += w[k]
        res["chunks"][K] = {"requests_per_sample": round(
            (tot["move_x"] + tot["move_yz"] + tot["chunk_end"]) / M, 4),
            **{k: round(v / M, 4) for k, v in tot.items()}, "per_level": per}
    Mh = a.hold_rays * a.samples
    xh = x[:Mh]
    res["segment_hold"] = {}
    for K in (256, 1024):
        cur = sum(sum(walk(lv, xh, K)[k] for k in ("move_x", "move_yz", "chunk_end"))
                  for lv in L)
        hold = sum(walk_segment_hold(lv, xh, K) for lv in L)
        res["segment_hold"][K] = {"rays": a.hold_rays,
                                  "current_requests_per_sample": round(cur / Mh, 4),
                                  "hold_requests_per_sample": round(hold / Mh, 4)}
    res["levels"] = [{k: (float(v) if isinstance(v, np.floating) else v) for k, v in lv.items()}
                     for lv in L]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
