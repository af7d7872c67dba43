"""``ray.tune.tune`` (reference: python/ray/tune/tune.py): the functional entry points."""

from ray_amd.tune.registry import run_experiments  # noqa: F401
from ray_amd.tune.tuner import run  # noqa: F401

__all__ = ["run", "run_experiments"]
