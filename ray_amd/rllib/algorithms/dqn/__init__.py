"""``ray.rllib.algorithms.dqn`` (reference: python/ray/rllib/algorithms/dqn/):
the algorithm and its config in ``dqn.py``, the learner in ``dqn_learner.py`` /
``torch/dqn_torch_learner.py``."""

from ray_amd.rllib.algorithms.dqn.dqn import DQN, DQNConfig  # noqa: F401
from ray_amd.rllib.algorithms.dqn.dqn_learner import DQNLearner  # noqa: F401

__all__ = ['DQN', 'DQNConfig', 'DQNLearner']
