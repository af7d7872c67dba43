"""``IMPALALearner`` (reference: python/ray/rllib/algorithms/impala/impala_learner.py). The PPO / IMPALA / APPO
losses share ray_amd's one torch Learner (core/learner/learner.py): the loss kind comes from
the algorithm config, and the whole SGD step runs as one captured HIP graph."""

from ray_amd.rllib.core.learner import Learner as IMPALALearner  # noqa: F401
