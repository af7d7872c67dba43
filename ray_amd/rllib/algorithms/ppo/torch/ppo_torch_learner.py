"""``PPOTorchLearner`` (reference: python/ray/rllib/algorithms/ppo/torch/ppo_torch_learner.py):
ray_amd's learners are torch learners; this is ``PPOLearner``."""

from ray_amd.rllib.algorithms.ppo.ppo_learner import PPOLearner as PPOTorchLearner  # noqa: F401
