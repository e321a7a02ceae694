"""Occupancy-grid sample culling for the Instant-NGP pipeline (BASELINE
configs[4]).

Beyond the reference: AtmoNR evaluates the field at every one of the N stratified samples
of every ray (instant_ngp.py:145,163-171) and has no occupancy structure (:27). This adds
the Instant-NGP occupancy grid as an opt-in (``InstantNGPPipeline(..., occupancy=...)`` or
the config key ``"occupancy_grid"``); without it the pipeline is the reference's uniform
sampler, which stays the parity default.

The grid covers the hash-grid domain [0,1] x [0,1] x [0, 1/alt_compress] with
gx x gy x gz cells. Each cell keeps a decayed running maximum of the field's density
(``density = max(decay * density, sigma(random point in the cell))``, refreshed every
``update_every`` training steps); a cell is occupied while that exceeds
min(``threshold``, mean cell density) — Instant-NGP's rule, so a scene whose learned
density is small everywhere still gets its thinnest cells culled; ``threshold`` is in
1/km, the pipeline's extinction unit. Every cell counts as occupied during the first
``warmup`` steps, and culling pauses while more than ``max_fraction`` of the cells are
occupied (compaction would then cost more than it saves). Samples in empty cells are culled before the hash grid and the MLPs
run: they keep sigma = 0 and colour 0, i.e. alpha = 0 in the composite, which is exact
for cells whose density really is zero and is Instant-NGP's approximation otherwise.
The composite, the loss and their gradients see the full dense (B, N) arrays.
"""

from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr


class OccupancyGrid:
    def __init__(self, resolution=(128, 128, 32), alt_compress: float = 8.0,
                 decay: float = 0.95, threshold: float = 0.01, update_every: int = 16,
                 warmup: int = 256, max_fraction: float = 0.9, device=None, seed: int = 0):
        self.res = tuple(int(r) for r in resolution)
        self.zmul = float(alt_compress)
        self.decay, self.threshold = float(decay), float(threshold)
        self.update_every, self.warmup = int(update_every), int(warmup)
        self.max_fraction = float(max_fraction)
        self.cell_fraction = 1.0  # occupied cells / all cells (host copy, per update)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        n = self.res[0] * self.res[1] * self.res[2]
        self.density = torch.zeros(n, device=self.device)
        self.occ = torch.ones(n, device=self.device, dtype=torch.uint8)
        self.steps = 0
        self.gen = torch.Generator(device=self.device).manual_seed(seed)
        self.last_fraction = 1.0  # kept samples / all samples of the last compaction

    @classmethod
    def from_config(cls, cfg: dict, alt_compress: float, device) -> "OccupancyGrid":
        return cls(resolution=cfg.get("resolution", (128, 128, 32)), alt_compress=alt_compress,
                   decay=cfg.get("decay", 0.95), threshold=cfg.get("threshold", 0.01),
                   update_every=cfg.get("update_every", 16), warmup=cfg.get("warmup", 256),
                   max_fraction=cfg.get("max_fraction", 0.9), device=device,
                   seed=cfg.get("seed", 0))

    @property
    def active(self) -> bool:
        """Culling is on once the warm-up steps are done and the grid is sparse enough."""
        return self.steps >= self.warmup and self.cell_fraction <= self.max_fraction

    def cell_points(self) -> torch.Tensor:
        """One uniformly jittered point per cell, in hash-grid coordinates (x fastest)."""
        gx, gy, gz = self.res
        iz, iy, ix = torch.meshgrid(torch.arange(gz, device=self.device),
                                    torch.arange(gy, device=self.device),
                                    torch.arange(gx, device=self.device), indexing="ij")
        cell = torch.stack([ix, iy, iz], dim=-1).reshape(-1, 3).float()
        u = torch.rand(cell.shape, device=self.device, generator=self.gen)
        p = (cell + u) / torch.tensor([gx, gy, gz], device=self.device, dtype=torch.float32)
        p[:, 2] = p[:, 2] / self.zmul
        return p

    @torch.no_grad()
    def update(self, density_fn) -> None:
        """Refresh the grid from ``density_fn(points (G,3)) -> sigma (G,)``; call once per
        training step (it acts every ``update_every`` steps)."""
        self.steps += 1
        if self.steps % self.update_every:
            return
        sigma = density_fn(self.cell_points()).reshape(-1).float()
        torch.maximum(self.density * self.decay, sigma, out=self.density)
        thr = torch.clamp(self.density.mean(), max=self.threshold)
        self.occ = (self.density > thr).to(torch.uint8)
        self.cell_fraction = float(self.occ.float().mean())  # one host read per update

    def set_occupancy(self, occ: torch.Tensor) -> None:
        """Install an occupancy mask (gx*gy*gz, x fastest; nonzero = occupied)."""
        self.occ = (occ.reshape(-1) != 0).to(torch.uint8).to(self.device)
        self.cell_fraction = float(self.occ.float().mean())

    def occupancy_fraction(self) -> float:
        return float(self.occ.float().mean())

    def compact(self, coords: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """coords (M,3) f32 ray-major -> (rows (K,) int32 ascending, coords[rows] (K,3)).
        One host read (the kept count) per call."""
        coords = coords.reshape(-1, 3).float().contiguous()
        M = coords.shape[0]
        dev = coords.device
        if not self.active:
            self.last_fraction = 1.0
            return torch.arange(M, device=dev, dtype=torch.int32), coords
        gx, gy, gz = self.res
        lib = _lib.load()
        nb = int(lib.anr_occupancy_n_blocks(M))
        s = _lib.stream(dev)
        counts = torch.empty(nb, device=dev, dtype=torch.int32)
        occ = self.occ.to(dev).contiguous()
        call("anr_occupancy_count", ptr(coords), M, ptr(occ), gx, gy, gz, self.zmul,
             ptr(counts), s)
        csum = counts.cumsum(0)
        K = int(csum[-1].item()) if nb else 0
        offsets = (csum - counts).contiguous()
        rows = torch.empty(K, device=dev, dtype=torch.int32)
        out = torch.empty(K, 3, device=dev, dtype=torch.float32)
        if K:
            call("anr_occupancy_compact", ptr(coords), M, ptr(occ), gx, gy, gz, self.zmul,
                 ptr(offsets), ptr(rows), ptr(out), s)
        self.last_fraction = K / max(1, M)
        return rows, out


def pipeline_density(pipe):
    """density_fn for OccupancyGrid.update: relu(pos_mlp(pos_encoder(p))[:, 0]) of an
    Instant-NGP pipeline at hash-grid points (the extract path without preprocessing)."""

    from .field import field_density, field_fused

    def fn(pts: torch.Tensor) -> torch.Tensor:
        if field_fused(pipe) and pipe.pos_encoder.dtype == torch.float16:
            return field_density(pipe, pts)
        out = pipe.pos_mlp(pipe.pos_encoder(pts))
        return torch.relu(out[:, 0].float())

    return fn

