from ray_amd.rllib.env import spaces  # noqa: F401
from ray_amd.rllib.env.envs import (CartPoleEnv, Env, PendulumEnv, RandomEnv,  # noqa: F401
                                    SyntheticAtariEnv, make_env, register_env)
from ray_amd.rllib.env.multi_agent_env import (MultiAgentCartPole, MultiAgentEnv,  # noqa: F401
                                              TicTacToe, TurnBasedGuess, make_multi_agent)
from ray_amd.rllib.env.env_context import EnvContext  # noqa: F401
from ray_amd.rllib.env.external_env import ExternalEnv  # noqa: F401
from ray_amd.rllib.env.vector_env import VectorEnv  # noqa: F401
from ray_amd.rllib.env.policy_client import PolicyClient  # noqa: F401
from ray_amd.rllib.env.policy_server_input import PolicyServerInput  # noqa: F401
from ray_amd.rllib.env.wrappers import (DMEnv, DMCEnv, GroupAgentsWrapper,  # noqa: F401
                                        ParallelPettingZooEnv, PettingZooEnv, Unity3DEnv)
from ray_amd.rllib.env.base_env import BaseEnv, ExternalMultiAgentEnv, RemoteBaseEnv  # noqa
from ray_amd.rllib.env.multi_agent_episode import MultiAgentEpisode  # noqa: F401,E402
from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode  # noqa: F401,E402
