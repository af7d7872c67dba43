"""ray_amd.train — distributed training (reference: python/ray/train/__init__.py)."""

from ray_amd.air.config import (CheckpointConfig, DatasetConfig, FailureConfig,  # noqa: F401
                                RunConfig, ScalingConfig)
from ray_amd.train._checkpoint import Checkpoint  # noqa: F401
from ray_amd.train._internal.session import (TrainContext, get_checkpoint,  # noqa: F401
                                             get_context, get_dataset_shard, report)
from ray_amd.train.backend import Backend, BackendConfig  # noqa: F401
from ray_amd.train.base_trainer import BaseTrainer  # noqa: F401
from ray_amd.train.data_parallel_trainer import (DataParallelTrainer,  # noqa: F401
                                                 TrainingFailedError)
from ray_amd.train.result import Result  # noqa: F401
from ray_amd.air.config import SyncConfig  # noqa: F401
from ray_amd.train.data_config import TRAIN_DATASET_KEY, DataConfig  # noqa: F401
from ray_amd.train.data_parallel_trainer import TrainingIterator  # noqa: F401

__all__ = ["BaseTrainer", "Checkpoint", "CheckpointConfig", "DataParallelTrainer", "FailureConfig", "Result",
           "RunConfig", "ScalingConfig", "TrainContext", "get_checkpoint", "get_context",
           "get_dataset_shard", "report", "Backend", "BackendConfig", "TrainingFailedError",
           "DatasetConfig", "DataConfig", "SyncConfig", "TrainingIterator", "TRAIN_DATASET_KEY"]
