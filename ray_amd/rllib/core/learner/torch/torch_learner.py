"""``ray.rllib.core.learner.torch.torch_learner`` (reference path): ``TorchLearner``."""

from ray_amd.rllib.core.learner.learner import TorchLearner  # noqa: F401
