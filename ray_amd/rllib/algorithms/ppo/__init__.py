"""``ray.rllib.algorithms.ppo`` (reference: python/ray/rllib/algorithms/ppo/):
the algorithm and its config in ``ppo.py``, the learner in ``ppo_learner.py`` /
``torch/ppo_torch_learner.py``."""

from ray_amd.rllib.algorithms.ppo.ppo import PPO, PPOConfig  # noqa: F401
from ray_amd.rllib.algorithms.ppo.ppo_learner import PPOLearner  # noqa: F401

__all__ = ['PPO', 'PPOConfig', 'PPOLearner']
