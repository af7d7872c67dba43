"""``DQNTorchLearner`` (reference: python/ray/rllib/algorithms/dqn/torch/dqn_torch_learner.py):
ray_amd's learners are torch learners; this is ``DQNLearner``."""

from ray_amd.rllib.algorithms.dqn.dqn_learner import DQNLearner as DQNTorchLearner  # noqa: F401
