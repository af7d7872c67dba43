"""``APPOTorchLearner`` (reference path)."""

from ray_amd.rllib.algorithms.appo.appo_learner import APPOLearner as APPOTorchLearner  # noqa: F401
