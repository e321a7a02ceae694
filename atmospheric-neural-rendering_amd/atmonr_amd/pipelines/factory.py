"""Pipeline registry — pipelines/factory.py:7-27 of the reference."""

from __future__ import annotations

from typing import Any

from .instant_ngp import InstantNGPPipeline
from .nerf import NeRFPipeline
from .pipeline import Pipeline

_PIPELINES: dict[str, type] = {"NeRF": NeRFPipeline, "InstantNGP": InstantNGPPipeline}


def register(name: str, cls: type) -> None:
    _PIPELINES[name] = cls


def get_pipeline(config: dict, dataset: Any, **kwargs) -> Pipeline:
    pipeline_type = config["type"]
    if pipeline_type not in _PIPELINES:
        raise NotImplementedError(f"Pipeline '{pipeline_type}' is unrecognized!")
    return _PIPELINES[pipeline_type](config, dataset, **kwargs)
