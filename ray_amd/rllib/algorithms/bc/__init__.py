"""reference import path ``ray.rllib.algorithms.bc``."""

from ray_amd.rllib.algorithms.marwil import BC, BCConfig  # noqa: F401

__all__ = ["BC", "BCConfig"]
