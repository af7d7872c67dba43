"""Run/scaling configuration dataclasses (reference: python/ray/air/config.py)."""

from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Callable


@dataclass
class ScalingConfig:
    num_workers: int = 1
    use_gpu: bool = False
    resources_per_worker: dict | None = None
    placement_strategy: str = "PACK"
    trainer_resources: dict | None = None
    accelerator_type: str | None = None

    @property
    def _resources_per_worker_not_none(self) -> dict:
        r = dict(self.resources_per_worker or {})
        if "CPU" not in r:
            r["CPU"] = 1
        if self.use_gpu and "GPU" not in r:
            r["GPU"] = 1
        if self.accelerator_type:  # workers only on nodes with that accelerator
            r[f"accelerator_type:{self.accelerator_type}"] = 0.001
        return {k: v for k, v in r.items() if v}

    @property
    def _trainer_bundle(self) -> dict | None:
        """trainer_resources: reserved for the run's coordinator (the driver-side trainer)
        as the placement group's first bundle; None when not requested."""
        tr = {k: v for k, v in (self.trainer_resources or {}).items() if v}
        return tr or None

    @property
    def num_gpus_per_worker(self):
        return self._resources_per_worker_not_none.get("GPU", 0)

    @property
    def num_cpus_per_worker(self):
        return self._resources_per_worker_not_none.get("CPU", 0)

    def as_placement_group_factory(self):
        workers = [self._resources_per_worker_not_none for _ in range(self.num_workers)]
        tb = self._trainer_bundle
        return ([tb] if tb else []) + workers

    @property
    def total_resources(self):
        out = {}
        for b in self.as_placement_group_factory():
            for k, v in b.items():
                out[k] = out.get(k, 0) + v
        return out


@dataclass
class FailureConfig:
    max_failures: int = 0
    fail_fast: bool = False


@dataclass
class CheckpointConfig:
    num_to_keep: int | None = None
    checkpoint_score_attribute: str | None = None
    checkpoint_score_order: str = "max"
    checkpoint_frequency: int = 0
    checkpoint_at_end: bool | None = None

    def __post_init__(self):
        if self.checkpoint_score_order not in ("max", "min"):
            raise ValueError("checkpoint_score_order must be 'max' or 'min'")
        if self.num_to_keep is not None and self.num_to_keep <= 0:
            raise ValueError("num_to_keep must be a positive integer or None")


@dataclass
class RunConfig:
    name: str | None = None
    storage_path: str | None = None
    storage_filesystem: Any = None
    failure_config: FailureConfig | None = None
    checkpoint_config: CheckpointConfig | None = None
    sync_config: Any = None
    verbose: int = 1
    stop: Any = None
    callbacks: list | None = None
    progress_reporter: Any = None
    log_to_file: Any = False

    def __post_init__(self):
        if self.storage_path is None:
            self.storage_path = os.environ.get("RAY_AMD_STORAGE",
                                               os.path.expanduser("~/ray_amd_results"))
        if self.failure_config is None:
            self.failure_config = FailureConfig()
        if self.checkpoint_config is None:
            self.checkpoint_config = CheckpointConfig()


@dataclass
class SyncConfig:
    """Checkpoint/artifact sync to ``RunConfig.storage_path`` (reference: train/
    _internal/syncer.py SyncConfig). A local or shared path is written in place (nothing
    to sync). With a non-local ``storage_filesystem`` Train workers upload checkpoints as
    they are reported, and Tune uploads its staged experiment directory (trial
    artifacts included) every ``sync_period`` seconds and at the end; uploads are
    synchronous, so ``sync_timeout`` and the artifact switches have nothing to bound."""

    sync_period: int = 300
    sync_timeout: int = 1800
    sync_artifacts: bool = False
    sync_artifacts_on_checkpoint: bool = True
    upload_dir: str | None = None
    syncer: object = None
    sync_on_checkpoint: bool = True

    def __post_init__(self):
        if self.upload_dir is not None:
            raise DeprecationWarning("SyncConfig(upload_dir) is deprecated: use "
                                     "RunConfig(storage_path=...)")


@dataclass
class DatasetConfig:
    fit: bool | None = None
    split: bool | None = None
    required: bool | None = None


field  # noqa: B018
Callable  # noqa: B018
