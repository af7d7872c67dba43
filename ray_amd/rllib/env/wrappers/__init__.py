"""Environment wrappers (reference: rllib/env/wrappers/).

``GroupAgentsWrapper`` runs here. The wrappers of third-party simulators — DeepMind
Control / dm_env, PettingZoo, Unity ML-Agents — need packages this image does not have;
constructing them raises ImportError naming the package."""

from ray_amd.rllib.env.wrappers.group_agents_wrapper import GroupAgentsWrapper  # noqa: F401


def _needs(pkg: str, what: str):
    class _Missing:
        def __init__(self, *a, **k):
            try:
                __import__(pkg)
            except ImportError as e:
                raise ImportError(f"{what} needs the '{pkg}' package, which is not "
                                  "installed") from e
            raise NotImplementedError(f"{what}: wrapper not implemented for {pkg}")

    _Missing.__name__ = what
    return _Missing


DMEnv = _needs("dm_env", "DMEnv")
DMCEnv = _needs("dm_control", "DMCEnv")
PettingZooEnv = _needs("pettingzoo", "PettingZooEnv")
ParallelPettingZooEnv = _needs("pettingzoo", "ParallelPettingZooEnv")
Unity3DEnv = _needs("mlagents_envs", "Unity3DEnv")
