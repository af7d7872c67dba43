"""``ray.tune.result_grid`` (reference: python/ray/tune/result_grid.py)."""

from ray_amd.tune.tuner import ResultGrid  # noqa: F401

__all__ = ["ResultGrid"]
