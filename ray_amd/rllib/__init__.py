"""ray_amd.rllib — reinforcement learning on MI355X (reference: rllib/)."""
from ray_amd.rllib.env.envs import register_env  # noqa: F401
