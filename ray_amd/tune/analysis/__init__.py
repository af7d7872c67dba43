"""reference: python/ray/tune/analysis/__init__.py."""

from ray_amd.tune.tuner import ExperimentAnalysis  # noqa: F401

__all__ = ["ExperimentAnalysis"]
