from ray_amd.rllib.env import spaces  # noqa: F401
from ray_amd.rllib.env.envs import (CartPoleEnv, Env, PendulumEnv, RandomEnv,  # noqa: F401
                                    SyntheticAtariEnv, make_env, register_env)
from ray_amd.rllib.env.multi_agent_env import (MultiAgentCartPole, MultiAgentEnv,  # noqa: F401
                                              TicTacToe, TurnBasedGuess, make_multi_agent)
