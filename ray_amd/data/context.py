"""``DataContext`` (reference: python/ray/data/context.py): the process-wide Ray Data
settings, snapshotted into each Dataset when it is created (``Dataset.context``).

Read by ray_amd's executor: ``target_max_block_size`` (oversized output blocks are cut,
data/_executor.py), ``execution_options`` (resource limits, locality, order), the
``use_push_based_shuffle`` / ``push_based_shuffle_merge_factor`` pair (Dataset.random_shuffle
and sort), ``enable_progress_bars`` and the free-form ``set_config`` entries. The remaining
attributes are the reference's knobs with its defaults, kept so configuration code that
sets them runs unchanged; ray_amd's block sizing and scheduling do not consult them."""

from __future__ import annotations

import copy
import threading
from typing import Any, Dict

from ray_amd.data._executor import ExecutionOptions

DEFAULT_TARGET_MAX_BLOCK_SIZE = 128 * 1024 * 1024
DEFAULT_SHUFFLE_TARGET_MAX_BLOCK_SIZE = 1024 * 1024 * 1024
DEFAULT_TARGET_MIN_BLOCK_SIZE = 1 * 1024 * 1024
ESTIMATED_SAFE_MEMORY_FRACTION = 0.25
MAX_SAFE_BLOCK_SIZE_FACTOR = 1.5
DEFAULT_STREAMING_READ_BUFFER_SIZE = 32 * 1024 * 1024
DEFAULT_ENABLE_PANDAS_BLOCK = True
DEFAULT_READ_OP_MIN_NUM_BLOCKS = 200
DEFAULT_ACTOR_PREFETCHER_ENABLED = False
DEFAULT_USE_PUSH_BASED_SHUFFLE = False
DEFAULT_SCHEDULING_STRATEGY = "SPREAD"
DEFAULT_SCHEDULING_STRATEGY_LARGE_ARGS = "DEFAULT"
DEFAULT_LARGE_ARGS_THRESHOLD = 50 * 1024 * 1024
DEFAULT_USE_POLARS = False
DEFAULT_EAGER_FREE = False
DEFAULT_ENABLE_PROGRESS_BARS = True
DEFAULT_MAX_ERRORED_BLOCKS = 0

_lock = threading.Lock()


class DataContext:
    _current = None

    def __init__(self):
        self.target_max_block_size = DEFAULT_TARGET_MAX_BLOCK_SIZE
        self.target_shuffle_max_block_size = DEFAULT_SHUFFLE_TARGET_MAX_BLOCK_SIZE
        self.target_min_block_size = DEFAULT_TARGET_MIN_BLOCK_SIZE
        self.streaming_read_buffer_size = DEFAULT_STREAMING_READ_BUFFER_SIZE
        self.enable_pandas_block = DEFAULT_ENABLE_PANDAS_BLOCK
        self.actor_prefetcher_enabled = DEFAULT_ACTOR_PREFETCHER_ENABLED
        self.use_push_based_shuffle = DEFAULT_USE_PUSH_BASED_SHUFFLE
        self.push_based_shuffle_merge_factor = 8
        self.scheduling_strategy = DEFAULT_SCHEDULING_STRATEGY
        self.scheduling_strategy_large_args = DEFAULT_SCHEDULING_STRATEGY_LARGE_ARGS
        self.large_args_threshold = DEFAULT_LARGE_ARGS_THRESHOLD
        self.use_polars = DEFAULT_USE_POLARS
        self.eager_free = DEFAULT_EAGER_FREE
        self.read_op_min_num_blocks = DEFAULT_READ_OP_MIN_NUM_BLOCKS
        self.enable_progress_bars = DEFAULT_ENABLE_PROGRESS_BARS
        self.enable_tensor_extension_casting = True
        self.enable_auto_log_stats = False
        self.verbose_stats_logs = False
        self.trace_allocations = False
        self.max_errored_blocks = DEFAULT_MAX_ERRORED_BLOCKS
        self.execution_options = ExecutionOptions()
        self._kv_configs: Dict[str, Any] = {}

    @classmethod
    def get_current(cls) -> "DataContext":
        with _lock:
            if cls._current is None:
                cls._current = DataContext()
            return cls._current

    @classmethod
    def _set_current(cls, context: "DataContext") -> None:
        """Install ``context`` as this process's current context (a worker adopting the
        driver's snapshot does this)."""
        cls._current = context

    def set_config(self, key: str, value: Any) -> None:
        self._kv_configs[key] = value

    def get_config(self, key: str, default: Any = None) -> Any:
        return self._kv_configs.get(key, default)

    def remove_config(self, key: str) -> None:
        self._kv_configs.pop(key, None)

    def copy(self) -> "DataContext":
        return copy.deepcopy(self)


DatasetContext = DataContext
