"""``ray.rllib.models.torch.torch_action_dist`` (reference path): the torch action
distributions, defined in ``models/action_dist.py``."""

from ray_amd.rllib.models.action_dist import (TorchCategorical, TorchDeterministic,  # noqa
                                              TorchDiagGaussian, TorchDistributionWrapper)
