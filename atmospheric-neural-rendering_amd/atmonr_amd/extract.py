"""Volume extraction — the loop of scripts/extract.py:180-211 over the L1C-style grid of
datasets/harp2_extract.py:71-187.

``GridExtractDataset`` builds the query points exactly as ``HARP2L1CExtractDataset``:
``sample_alt = arange(min_alt, max_alt + alt_step / 2, alt_step)`` (f32, the torch default
dtype), every horizontal grid cell repeated over the altitudes, converted to WGS-84
Cartesian in f64 (``horizontal_to_cartesian``). The horizontal grid is the dataset's
pixel lat/lon (the L1C grid needs the NASA download, absent offline) or any (H, W) lat/lon
the caller passes (voxel-grid mode).

``extract_volume`` runs the reference loop: batches of ``batch_size`` columns
(``batch_size · n_alt`` points, unshuffled), ``pts = (xyz - offset) / scale`` in f64,
``sigma[idx] = pipeline.extract(pts) / scale``. On MI355X the points stay in HBM, the
f64 preprocessor runs as one kernel (anr_preprocess_points_f64) and the hash encoder +
density MLP as the same kernels training uses; the host only slices index ranges.
``dump`` writes an .npz with the reference's netCDF variables (netCDF4 is not installed).
"""

from __future__ import annotations

import inspect
from pathlib import Path

import numpy as np
import torch

from .batch_loader import BatchLoader
from .geospatial.wgs_84 import horizontal_to_cartesian


class GridExtractDataset:
    def __init__(self, dataset, alt_step: float = 250.0, min_alt: float | None = None,
                 max_alt: float | None = None, lat: torch.Tensor | None = None,
                 lon: torch.Tensor | None = None) -> None:
        self.dataset = dataset
        self.device = dataset.device
        self.alt_step = alt_step
        self.min_alt = 0 if min_alt is None else min_alt
        self.max_alt = dataset.config["ray_origin_height"] if max_alt is None else max_alt
        self.sample_alt = torch.arange(self.min_alt, self.max_alt + self.alt_step / 2,
                                       self.alt_step).to(self.device)
        if lat is None:
            H, W = dataset.img_shp
            lat = dataset.lat[:, 0].view(H, W)
            lon = dataset.lon[:, 0].view(H, W)
        self.shp = tuple(lat.shape)
        A = self.sample_alt.shape[0]
        self.lat = lat[:, :, None].repeat(1, 1, A).to(self.device)
        self.lon = lon[:, :, None].repeat(1, 1, A).to(self.device)
        alt = self.sample_alt[None, None].repeat(self.lat.shape[0], self.lat.shape[1], 1)
        xyz = torch.stack(list(horizontal_to_cartesian(
            self.lat.double(), self.lon.double(), alt.double())), dim=-1)
        self.xyz = xyz.view(-1, 3)
        self.idx = torch.arange(self.xyz.shape[0], device=self.device, dtype=torch.int64)

    def __len__(self) -> int:
        return int(self.xyz.shape[0])

    def __getbatch__(self, idx: torch.Tensor) -> dict[str, torch.Tensor]:
        return {"xyz": self.xyz[idx], "idx": self.idx[idx]}

    __getitem__ = __getbatch__

    def dump(self, path: Path | str, sigma: torch.Tensor) -> None:
        """Variables of _extract_to_netCDF (harp2_extract.py:429-596) as an .npz."""
        A = self.sample_alt.shape[0]
        np.savez(path,
                 extinction=sigma.view(*self.shp, A, -1).cpu().numpy(),
                 latitude=self.lat[:, :, 0].cpu().numpy(),
                 longitude=self.lon[:, :, 0].cpu().numpy(),
                 sample_alt=self.sample_alt.cpu().numpy(),
                 xyz=self.xyz.view(*self.shp, A, 3).cpu().numpy())


def _extract(pipeline, pts, run_length):
    """pipeline.extract with the column run length when the pipeline takes the hint (the
    batches are whole columns of ``run_length`` altitudes)."""
    if "run_length" in inspect.signature(pipeline.extract).parameters:
        return pipeline.extract(pts, run_length=run_length)
    return pipeline.extract(pts)


def extract_volume(pipeline, dataset, extract_ds: GridExtractDataset, batch_size: int = 32768,
                   num_bands: int = 1) -> torch.Tensor:
    """scripts/extract.py:183-209: extinction (n_points, num_bands) in 1/m."""
    A = int(extract_ds.sample_alt.shape[0])
    loader = BatchLoader(extract_ds, batch_size=batch_size * A, shuffle=False)
    sigma = torch.zeros((len(extract_ds), num_bands), device=extract_ds.device)
    offset = torch.as_tensor(dataset.offset, dtype=torch.float64, device=extract_ds.device)
    with torch.no_grad():
        for batch in loader:
            pts = (batch["xyz"] - offset) / dataset.scale
            sigma[batch["idx"]] = _extract(pipeline, pts, A).to(dtype=sigma.dtype) / dataset.scale
    return sigma
