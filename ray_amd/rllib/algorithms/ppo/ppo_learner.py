"""``PPOLearner`` (reference: python/ray/rllib/algorithms/ppo/ppo_learner.py). The PPO / IMPALA / APPO
losses share ray_amd's one torch Learner (core/learner/learner.py): the loss kind comes from
the algorithm config, and the whole SGD step runs as one captured HIP graph."""

from ray_amd.rllib.core.learner import Learner as PPOLearner  # noqa: F401
