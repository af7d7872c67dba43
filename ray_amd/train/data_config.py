"""``DataConfig``: which Train datasets are sharded across workers (reference:
python/ray/train/_internal/data_config.py). ``datasets_to_split="all"`` (default) gives
every worker an equal ``streaming_split`` shard of each dataset; datasets not listed are
handed whole (as an iterator) to every worker."""

from __future__ import annotations

from typing import List, Literal, Optional, Union

TRAIN_DATASET_KEY = "train"


class DataConfig:
    def __init__(self, datasets_to_split: Union[Literal["all"], List[str]] = "all",
                 execution_options=None, enable_shard_locality: bool = True):
        if not (datasets_to_split == "all" or isinstance(datasets_to_split, (list, tuple))):
            raise TypeError("datasets_to_split must be 'all' or a list of dataset names, got "
                            f"{datasets_to_split!r}")
        self.datasets_to_split = datasets_to_split if datasets_to_split == "all" else \
            list(datasets_to_split)
        self.execution_options = execution_options
        self.enable_shard_locality = enable_shard_locality

    @staticmethod
    def default_ingest_options():
        from ray_amd.data import ExecutionOptions

        return ExecutionOptions()

    def __repr__(self):
        return f"DataConfig(datasets_to_split={self.datasets_to_split!r})"
