"""``ray.rllib.core.rl_module.marl_module`` (reference path): the multi-agent module
container and its spec (``MultiRLModule`` in checkpoint.py, ``MultiRLModuleSpec`` in
rl_module.py)."""

from ray_amd.rllib.core.rl_module.checkpoint import MultiRLModule  # noqa: F401
from ray_amd.rllib.core.rl_module.rl_module import MultiRLModuleSpec  # noqa: F401

MultiAgentRLModule = MultiRLModule
MultiAgentRLModuleSpec = MultiRLModuleSpec
