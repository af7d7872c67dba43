"""``APPO`` / ``APPOConfig`` (reference: python/ray/rllib/algorithms/appo/appo.py): IMPALA's
asynchronous pipeline with the clipped surrogate loss (algorithms/impala/impala.py)."""

from ray_amd.rllib.algorithms.impala.impala import APPO, APPOConfig  # noqa: F401
