"""reference import path ``ray.rllib.algorithms.appo``."""

from ray_amd.rllib.algorithms.impala import APPO, APPOConfig  # noqa: F401

__all__ = ["APPO", "APPOConfig"]
