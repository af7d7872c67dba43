"""``PPOTorchRLModule`` (reference: python/ray/rllib/algorithms/ppo/torch/ppo_torch_rl_module.py)."""

from ray_amd.rllib.core.rl_module.default import RLModule as PPOTorchRLModule  # noqa: F401
