"""``DQNLearner`` (reference: python/ray/rllib/algorithms/dqn/dqn_learner.py)."""

from ray_amd.rllib.algorithms.dqn.dqn import DQNLearner as DQNLearner  # noqa: F401
