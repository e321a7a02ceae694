"""Memory-side atomic requests of one hash-grid backward launch, counted from its inputs.

hashgrid_bwd_v2_kernel (csrc/hashgrid.hip) walks each chunk of K consecutive samples with
4 lanes per level (x-offset b, feature f); a lane holds the f32 gradient of the NC = 4
(y, z) corners of the current cell and issues one no-return f32 atomic per corner that
leaves (cell move) and per corner at the chunk end. The hardware turns one wave
instruction into one 64-B request per distinct 64-B segment its active lanes touch
(MI355X_MICROARCH.md "Global float atomics"); the lanes of one level touch entries x and
x+1 of one (y, z) row, 2 x 8 B, so a leaving corner costs 1 request, or 2 when the pair
straddles a segment edge. This counts exactly those requests for given coordinates: the
same cells (fmaf(scale, x, 0.5) in f32, floor), chunking (the launch's K) and corner
indexing (tcnn's dense stride / XOR-prime hash) as the kernel.

Checked against rocprofv3 TCC_EA0_ATOMIC_sum on the bench launch: 2.5086 vs 2.508
requests per sample (profiles/r04_hash_bwd_requests.json, profiles/pmc_traffic.json).
bench.py counts the benched batch this way in its untimed phase (the roofline's request
count is then measured from the run's own coordinates, not read from a stored PMC entry).
"""

from __future__ import annotations


import torch

PRIMES = (1, 2654435761, 805459861)
U32 = 0xFFFFFFFF


def bwd_chunk(M: int) -> int:
    """pick_chunk_v2 (csrc/hashgrid.hip): samples per wave of the v2 backward, asked of
    the library itself (anr_hashgrid_bwd_chunk, ANR_HASH_KB included)."""
    from atmonr_amd import _lib

    return int(_lib.load().anr_hashgrid_bwd_chunk(int(M)))


def level_geometry(desc) -> list[dict]:
    """Per level: scale (f32), res, T, table offset (entries) from an anr_hashgrid_desc."""
    out = []
    for lv in range(desc.n_levels):
        T = int(desc.offsets[lv + 1] - desc.offsets[lv])
        res = int(desc.resolutions[lv])
        out.append({"scale": float(desc.scales[lv]), "res": res, "T": T,
                    "offset": int(desc.offsets[lv]), "hashed": res ** desc.n_dims > T})
    return out


def _index(lv: dict, g: torch.Tensor) -> torch.Tensor:
    """Entry index within the level of lattice points g (..., 3) int64 (grid_index)."""
    if lv["hashed"]:
        h = torch.zeros(g.shape[:-1], dtype=torch.int64, device=g.device)
        for d in range(g.shape[-1]):
            h ^= (g[..., d] * PRIMES[d]) & U32
        return h & (lv["T"] - 1)
    s = g[..., 0]
    st = lv["res"]
    for d in range(1, g.shape[-1]):
        s = s + g[..., d] * st
        st *= lv["res"]
    return (s & U32) % lv["T"]


def _pair_requests(lv: dict, c: torch.Tensor, cy: int, cz: int) -> torch.Tensor:
    g0 = c.clone()
    g0[:, 1] += cy
    if g0.shape[1] > 2:
        g0[:, 2] += cz
    g1 = g0.clone()
    g1[:, 0] += 1
    s0 = (lv["offset"] + _index(lv, g0)) >> 3  # 64-B segment of the 8-B f32 pair
    s1 = (lv["offset"] + _index(lv, g1)) >> 3
    return 1 + (s0 != s1).to(torch.int64)


def count(x: torch.Tensor, desc, K: int | None = None, by_cause: bool = False):
    """Requests of anr_hashgrid_bwd over coordinates x (M, D) f32 (the v2 kernel: F = 2,
    up to 16 levels). Returns the total, or {cause: count} with ``by_cause``."""
    x = x.reshape(-1, x.shape[-1]).float()
    M, D = x.shape
    K = bwd_chunk(M) if K is None else K
    pos_in = x.double()
    chunk = torch.arange(M, device=x.device) // K
    first = torch.ones(M, dtype=torch.bool, device=x.device)
    first[1:] = chunk[1:] != chunk[:-1]
    last = torch.ones(M, dtype=torch.bool, device=x.device)
    last[:-1] = first[1:]
    rows = [(cy, cz) for cz in ((0, 1) if D == 3 else (0,)) for cy in (0, 1)]
    tot = {"move_x": 0, "move_yz": 0, "chunk_end": 0}
    for lv in level_geometry(desc):
        # fmaf(scale, x, 0.5): the f64 product of two f32 values is exact, one rounding
        pos = (lv["scale"] * pos_in + 0.5).float()
        cell = torch.floor(pos).to(torch.int64)
        moved = torch.zeros(M, dtype=torch.bool, device=x.device)
        moved[1:] = (cell[1:] != cell[:-1]).any(dim=1)
        moved &= ~first
        t = torch.nonzero(moved).squeeze(1)
        old, new = cell[t - 1], cell[t]
        keepx = old[:, 0] == new[:, 0]
        dl = old - new
        for cy, cz in rows:
            leaves = ~keepx | ((cy + dl[:, 1]) < 0) | ((cy + dl[:, 1]) > 1)
            if D == 3:
                leaves |= ((cz + dl[:, 2]) < 0) | ((cz + dl[:, 2]) > 1)
            r = _pair_requests(lv, old, cy, cz)
            tot["move_x"] += int(r[leaves & ~keepx].sum())
            tot["move_yz"] += int(r[leaves & keepx].sum())
            tot["chunk_end"] += int(_pair_requests(lv, cell[last], cy, cz).sum())
    if by_cause:
        return tot
    return sum(tot.values())
