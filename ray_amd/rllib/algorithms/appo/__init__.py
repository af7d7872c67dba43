"""``ray.rllib.algorithms.appo`` (reference: python/ray/rllib/algorithms/appo/)."""

from ray_amd.rllib.algorithms.appo.appo import APPO, APPOConfig  # noqa: F401
from ray_amd.rllib.algorithms.appo.appo_learner import APPOLearner  # noqa: F401

__all__ = ["APPO", "APPOConfig", "APPOLearner"]
