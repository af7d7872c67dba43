"""``MARWILTorchLearner`` (reference: python/ray/rllib/algorithms/marwil/torch/marwil_torch_learner.py):
ray_amd's learners are torch learners; this is ``MARWILLearner``."""

from ray_amd.rllib.algorithms.marwil.marwil_learner import MARWILLearner as MARWILTorchLearner  # noqa: F401
