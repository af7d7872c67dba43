"""``IMPALATorchLearner`` (reference: python/ray/rllib/algorithms/impala/torch/impala_torch_learner.py):
ray_amd's learners are torch learners; this is ``IMPALALearner``."""

from ray_amd.rllib.algorithms.impala.impala_learner import IMPALALearner as IMPALATorchLearner  # noqa: F401
