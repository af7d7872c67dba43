"""``ray.rllib.core.rl_module.multi_rl_module`` (newer reference path)."""

from ray_amd.rllib.core.rl_module.checkpoint import MultiRLModule  # noqa: F401
from ray_amd.rllib.core.rl_module.rl_module import MultiRLModuleSpec  # noqa: F401
