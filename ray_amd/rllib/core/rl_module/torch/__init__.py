"""reference path: ``rllib.core.rl_module.torch.TorchRLModule``."""
from ray_amd.rllib.core.rl_module.rl_module import TorchRLModule  # noqa: F401

TorchRLModule = TorchRLModule
