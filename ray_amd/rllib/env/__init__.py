from ray_amd.rllib.env import spaces  # noqa: F401
from ray_amd.rllib.env.envs import (CartPoleEnv, Env, PendulumEnv, RandomEnv,  # noqa: F401
                                    SyntheticAtariEnv, make_env, register_env)
