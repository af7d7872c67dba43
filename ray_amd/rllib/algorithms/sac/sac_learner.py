"""``SACLearner`` (reference: python/ray/rllib/algorithms/sac/sac_learner.py)."""

from ray_amd.rllib.algorithms.sac.sac import SACLearner as SACLearner  # noqa: F401
