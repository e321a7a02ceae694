"""Pipeline base class — the drop-in boundary of src/atmonr/pipelines/pipeline.py:10-92.

A pipeline is constructed as ``(config, dataset)`` and exposes ``send_tensors_to``,
``get_optimizer``, ``forward(ray_batch) -> dict``, ``extract(pts)``, ``compute_loss``,
``state_dict`` / ``load_state_dict`` and ``train`` / ``eval``, exactly as the reference.
"""

from __future__ import annotations

import warnings
from typing import Any, Mapping

import torch
from torch.optim import Optimizer


class Pipeline:
    def __init__(self, config: dict, dataset: Any) -> None:
        # pipeline.py:30-60
        self.ray_origin_height = dataset.config["ray_origin_height"]
        assert not (config["point_preprocessor"] == "horizontal" and config["include_height"])
        enc = config.get("encoder")
        if (
            not config["point_preprocessor"]
            and enc is not None
            and isinstance(enc["L_x"], list)
            and not all(n == enc["L_x"][0] for n in enc["L_x"])
        ):
            warnings.warn(
                "Are you sure you want to use a variable encoding dimension for "
                "non-transformed coordinates?"
            )
        self.device = -1
        self.config = config
        self.scale = dataset.scale
        self.offset = dataset.offset
        if self.config["point_preprocessor"]:
            self.point_preprocessor = dataset.get_point_preprocessor(
                self.config["point_preprocessor"]
            )
        else:
            self.point_preprocessor = None

    def send_tensors_to(self, device: int) -> None:
        raise NotImplementedError

    def get_optimizer(self, config: dict) -> Optimizer:
        raise NotImplementedError

    def forward(self, ray_batch: Mapping[str, torch.Tensor]) -> dict[str, torch.Tensor]:
        raise NotImplementedError

    def extract(self, pts: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def compute_loss(self, ray_batch: Mapping[str, torch.Tensor],
                     results: dict[str, torch.Tensor]) -> torch.Tensor:
        raise NotImplementedError

    def state_dict(self) -> Mapping[str, Mapping[str, Any]]:
        raise NotImplementedError

    def load_state_dict(self, state_dict: dict) -> None:
        raise NotImplementedError

    def train(self) -> None:
        raise NotImplementedError

    def eval(self) -> None:
        raise NotImplementedError
