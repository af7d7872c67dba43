"""Old-stack execution helpers (reference: rllib/execution/{rollout_ops,train_ops}.py)."""

from ray_amd.rllib.execution.rollout_ops import synchronous_parallel_sample  # noqa: F401
from ray_amd.rllib.execution.train_ops import train_one_step  # noqa: F401
