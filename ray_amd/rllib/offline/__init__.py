"""Offline RL data and evaluation (reference: rllib/offline/).

* ``io``: fragment-JSON and transition-Parquet writers, ``read_offline_dataset`` (a
  ray_amd.data Dataset of transition rows with episode ids).
* ``offline_data``: ``OfflineData`` — returns-to-go per episode, a shuffled epoch stream
  for one learner, ``streaming_split`` shards for learner actors.
* ``estimators``: off-policy estimation (IS, WIS, DM, DR over an FQE Q-model) wired to
  ``AlgorithmConfig.evaluation(off_policy_estimation_methods=...)``.
"""

from .io import (JsonReader, JsonWriter, ParquetWriter, discounted_returns,
                 fragment_to_transitions, read_offline_dataset)
from .offline_data import OfflineData, add_returns, iterate_forever
from .io_context import (DatasetReader, DatasetWriter, InputReader, IOContext,  # noqa: F401
                         MixedInput, NoopOutput, OutputWriter, ShuffledInput,
                         get_dataset_and_shards, get_offline_io_resource_bundles)
from .estimators import (DirectMethod, DoublyRobust, FQETorchModel, ImportanceSampling,
                         OfflineEvaluator, OffPolicyEstimator, WeightedImportanceSampling)

__all__ = ["DatasetReader", "DatasetWriter", "InputReader", "IOContext", "MixedInput",
           "NoopOutput", "OutputWriter", "ShuffledInput", "get_dataset_and_shards",
           "get_offline_io_resource_bundles", "DirectMethod", "DoublyRobust", "FQETorchModel", "ImportanceSampling",
           "JsonReader", "JsonWriter", "OfflineData", "OfflineEvaluator",
           "OffPolicyEstimator", "ParquetWriter", "WeightedImportanceSampling",
           "add_returns", "discounted_returns", "fragment_to_transitions", "iterate_forever",
           "read_offline_dataset"]
