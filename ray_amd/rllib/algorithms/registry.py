"""Algorithm registry (reference: rllib/algorithms/registry.py)."""


def _algos():
    from ray_amd.rllib.algorithms.dqn import DQN, DQNConfig
    from ray_amd.rllib.algorithms.impala import APPO, IMPALA, APPOConfig, IMPALAConfig
    from ray_amd.rllib.algorithms.ppo import PPO, PPOConfig
    from ray_amd.rllib.algorithms.cql import CQL, CQLConfig
    from ray_amd.rllib.algorithms.marwil import BC, MARWIL, BCConfig, MARWILConfig
    from ray_amd.rllib.algorithms.sac import SAC, SACConfig
    from ray_amd.rllib.algorithms.dreamerv3 import DreamerV3, DreamerV3Config

    return {"PPO": (PPO, PPOConfig), "IMPALA": (IMPALA, IMPALAConfig),
            "APPO": (APPO, APPOConfig), "DQN": (DQN, DQNConfig), "SAC": (SAC, SACConfig),
            "CQL": (CQL, CQLConfig), "MARWIL": (MARWIL, MARWILConfig), "BC": (BC, BCConfig),
            "DreamerV3": (DreamerV3, DreamerV3Config)}


def get_algorithm_class(name: str):
    return _algos()[name][0]


def get_config_class(cls):
    for a, c in _algos().values():
        if a is cls:
            return c
    raise KeyError(cls)


ALGORITHMS = property(_algos)
