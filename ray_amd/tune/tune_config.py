"""``ray.tune.tune_config`` (reference: python/ray/tune/tune_config.py)."""

from ray_amd.tune.tuner import ResumeConfig, TuneConfig  # noqa: F401

__all__ = ["TuneConfig", "ResumeConfig"]
