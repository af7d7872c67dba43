"""``DefaultPPOTorchRLModule`` (reference path)."""

from ray_amd.rllib.core.rl_module.default import RLModule as DefaultPPOTorchRLModule  # noqa: F401
