"""``ray.rllib.core.rl_module.torch.torch_rl_module`` (reference path)."""

from ray_amd.rllib.core.rl_module.rl_module import TorchRLModule  # noqa: F401
