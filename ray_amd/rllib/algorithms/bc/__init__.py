"""``ray.rllib.algorithms.bc`` (reference: python/ray/rllib/algorithms/bc/)."""

from ray_amd.rllib.algorithms.bc.bc import BC, BCConfig  # noqa: F401

__all__ = ["BC", "BCConfig"]
