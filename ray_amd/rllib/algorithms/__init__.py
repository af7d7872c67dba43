from ray_amd.rllib.algorithms.algorithm import Algorithm  # noqa: F401
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig  # noqa: F401
from ray_amd.rllib.algorithms.dqn import DQN, DQNConfig  # noqa: F401
from ray_amd.rllib.algorithms.impala import APPO, IMPALA, APPOConfig, IMPALAConfig  # noqa: F401
from ray_amd.rllib.algorithms.ppo import PPO, PPOConfig  # noqa: F401
from ray_amd.rllib.algorithms.sac import SAC, SACConfig  # noqa: F401
from ray_amd.rllib.algorithms.cql import CQL, CQLConfig  # noqa: F401
from ray_amd.rllib.algorithms.marwil import BC, MARWIL, BCConfig, MARWILConfig  # noqa: F401
from ray_amd.rllib.algorithms.dreamerv3 import DreamerV3, DreamerV3Config  # noqa: F401
