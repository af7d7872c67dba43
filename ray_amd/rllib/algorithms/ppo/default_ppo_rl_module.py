"""``DefaultPPORLModule`` (reference: python/ray/rllib/algorithms/ppo/
default_ppo_rl_module.py): ray_amd's default actor-critic module (MLP or Nature-CNN encoder,
policy and value heads; core/rl_module/default.py)."""

from ray_amd.rllib.core.rl_module.default import RLModule as DefaultPPORLModule  # noqa: F401
