"""Environment checker (reference: rllib/utils/pre_checks/env.py check_env): the env's
spaces exist, ``reset`` returns ``(obs, infos)`` and ``step`` the 5-tuple, and the
observations lie in the observation space."""

from __future__ import annotations

import numpy as np


def _contains(space, obs) -> bool:
    try:
        return bool(space.contains(obs))
    except Exception:  # noqa: BLE001 - spaces without contains()
        return True


def check_env(env, config=None) -> None:
    from ray_amd.rllib.env.multi_agent_env import MultiAgentEnv

    if isinstance(env, MultiAgentEnv):
        obs, infos = env.reset()
        if not isinstance(obs, dict):
            raise ValueError("MultiAgentEnv.reset() must return a dict of observations")
        acts = {aid: env.action_space.sample() if not hasattr(env, "get_action_space") else
                env.get_action_space(aid).sample() for aid in obs}
        out = env.step(acts)
        if len(out) != 5:
            raise ValueError("MultiAgentEnv.step() must return (obs, rewards, terminateds, "
                             "truncateds, infos)")
        if "__all__" not in out[2]:
            raise ValueError("terminateds must contain the '__all__' key")
        return
    for attr in ("observation_space", "action_space"):
        if getattr(env, attr, None) is None:
            raise ValueError(f"env has no {attr}")
    r = env.reset()
    if not (isinstance(r, tuple) and len(r) == 2):
        raise ValueError("reset() must return (observation, infos) (gymnasium API)")
    obs, infos = r
    if not isinstance(infos, dict):
        raise ValueError("reset() infos must be a dict")
    if not _contains(env.observation_space, obs):
        raise ValueError(f"reset() observation {np.asarray(obs).shape} is not in "
                         f"{env.observation_space}")
    out = env.step(env.action_space.sample())
    if not (isinstance(out, tuple) and len(out) == 5):
        raise ValueError("step() must return (obs, reward, terminated, truncated, infos)")
    obs, rew, term, trunc, infos = out
    if not _contains(env.observation_space, obs):
        raise ValueError("step() observation is not in the observation space")
    if not np.isscalar(rew) and np.asarray(rew).shape != ():
        raise ValueError(f"reward must be a scalar, got {type(rew)}")
    if not isinstance(term, (bool, np.bool_)) or not isinstance(trunc, (bool, np.bool_)):
        raise ValueError("terminated / truncated must be bools")
