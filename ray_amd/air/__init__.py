"""ray_amd.air — shared configs (reference: python/ray/air)."""
from ray_amd.air.config import (CheckpointConfig, DatasetConfig, FailureConfig,  # noqa: F401
                                RunConfig, ScalingConfig)
from ray_amd.train.result import Result  # noqa: F401
from ray_amd.air.data_batch_type import DataBatchType  # noqa: F401,E402
from ray_amd.air.execution.resources import AcquiredResources, ResourceRequest  # noqa: F401,E402
