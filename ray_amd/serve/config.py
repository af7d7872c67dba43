"""Serve configuration models (reference: python/ray/serve/config.py).

``AutoscalingConfig`` is validated with pydantic like the reference's and turned into the
plain dict the controller's autoscaling loop reads (``_controller.ServeController
._autoscale``); only the fields the user set travel, so the controller's own defaults
apply to the rest."""

from __future__ import annotations

from enum import Enum
from typing import Any, Optional

from pydantic import BaseModel, Field, model_validator

from ray_amd.serve.api import HTTPOptions, gRPCOptions  # noqa: F401


class AutoscalingConfig(BaseModel):
    min_replicas: int = Field(default=1, ge=0)
    initial_replicas: Optional[int] = Field(default=None, ge=0)
    max_replicas: int = Field(default=1, gt=0)
    target_ongoing_requests: Optional[float] = Field(default=None, gt=0)
    # deprecated alias of target_ongoing_requests
    target_num_ongoing_requests_per_replica: float = Field(default=1.0, gt=0)
    metrics_interval_s: float = Field(default=10.0, gt=0)
    look_back_period_s: float = Field(default=30.0, gt=0)
    smoothing_factor: float = Field(default=1.0, gt=0)
    upscale_smoothing_factor: Optional[float] = Field(default=None, gt=0)
    downscale_smoothing_factor: Optional[float] = Field(default=None, gt=0)
    upscaling_factor: Optional[float] = Field(default=None, gt=0)
    downscaling_factor: Optional[float] = Field(default=None, gt=0)
    downscale_delay_s: float = Field(default=600.0, ge=0)
    upscale_delay_s: float = Field(default=30.0, ge=0)
    # the decision function (serve/autoscaling_policy.py): a callable or an import path;
    # None = replica_queue_length_autoscaling_policy
    policy: Optional[Any] = None

    @model_validator(mode="after")
    def _replica_bounds(self):
        if self.max_replicas < self.min_replicas:
            raise ValueError(f"max_replicas ({self.max_replicas}) must be greater than or "
                             f"equal to min_replicas ({self.min_replicas})!")
        if self.initial_replicas is not None:
            if self.initial_replicas < self.min_replicas:
                raise ValueError(f"min_replicas ({self.min_replicas}) must be less than or "
                                 f"equal to initial_replicas ({self.initial_replicas})!")
            if self.initial_replicas > self.max_replicas:
                raise ValueError(f"max_replicas ({self.max_replicas}) must be greater than "
                                 f"or equal to initial_replicas ({self.initial_replicas})!")
        return self

    @classmethod
    def default(cls) -> "AutoscalingConfig":
        return cls(target_ongoing_requests=2.0, min_replicas=1, max_replicas=100)

    def get_target_ongoing_requests(self) -> float:
        if self.target_ongoing_requests is not None:
            return self.target_ongoing_requests
        return self.target_num_ongoing_requests_per_replica

    def get_upscaling_factor(self) -> float:
        return self.upscaling_factor or self.upscale_smoothing_factor or self.smoothing_factor

    def get_downscaling_factor(self) -> float:
        return (self.downscaling_factor or self.downscale_smoothing_factor or
                self.smoothing_factor)

    def to_controller_dict(self) -> dict:
        d = self.model_dump(exclude_unset=True)
        d["target_ongoing_requests"] = self.get_target_ongoing_requests()
        d.setdefault("min_replicas", self.min_replicas)
        d.setdefault("max_replicas", self.max_replicas)
        if "upscaling_factor" in d or "upscale_smoothing_factor" in d or \
                "smoothing_factor" in d:
            d["upscaling_factor"] = self.get_upscaling_factor()
        if "downscaling_factor" in d or "downscale_smoothing_factor" in d or \
                "smoothing_factor" in d:
            d["downscaling_factor"] = self.get_downscaling_factor()
        return d


def normalize_autoscaling_config(cfg) -> Optional[dict]:
    """AutoscalingConfig | dict | None -> the controller's dict (validated)."""
    if cfg is None:
        return None
    if isinstance(cfg, AutoscalingConfig):
        return cfg.to_controller_dict()
    if isinstance(cfg, dict):
        if "_policy" in cfg:  # the reference's private spelling
            cfg = dict(cfg)
            cfg["policy"] = cfg.pop("_policy")
        known = set(AutoscalingConfig.model_fields)
        unknown = set(cfg) - known
        if unknown:
            raise ValueError(f"unknown autoscaling_config keys: {sorted(unknown)}")
        return AutoscalingConfig(**cfg).to_controller_dict()
    raise TypeError(f"autoscaling_config must be a dict or AutoscalingConfig, got {cfg!r}")


class DeploymentMode(str, Enum):
    NoServer = "NoServer"
    HeadOnly = "HeadOnly"
    EveryNode = "EveryNode"


class ProxyLocation(str, Enum):
    """Where HTTP proxies run: ``HeadOnly`` one on the head node, ``EveryNode`` one per
    alive node (started / stopped by the controller as nodes join and leave),
    ``Disabled`` none."""
    Disabled = "Disabled"
    HeadOnly = "HeadOnly"
    EveryNode = "EveryNode"
