"""``BaseEnv`` (reference: python/ray/rllib/env/base_env.py): the old API stack's
vectorized, multi-agent, asynchronous env interface.

``poll()`` returns the ready data of every sub-env as nested dicts
``env_id -> agent_id -> value`` (observations, rewards, terminateds, truncateds, infos,
off-policy actions); ``send_actions`` takes the same nesting; ``try_reset(env_id)``
restarts one sub-env. ``convert_to_base_env`` wraps gym-style single-agent envs, vectors
of them, MultiAgentEnvs and ExternalEnvs. ray_amd's EnvRunners step envs in lock-step
directly; this interface is for code written against the old stack."""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

_DUMMY_AGENT_ID = "agent0"


class BaseEnv:
    def poll(self) -> Tuple[dict, dict, dict, dict, dict, dict]:
        raise NotImplementedError

    def send_actions(self, action_dict: dict) -> None:
        raise NotImplementedError

    def try_reset(self, env_id=None, *, seed=None, options=None):
        return None, None

    def try_restart(self, env_id=None) -> None:
        self.try_reset(env_id)

    def get_sub_environments(self, as_dict: bool = False):
        return {} if as_dict else []

    def get_agent_ids(self):
        return {_DUMMY_AGENT_ID}

    def stop(self) -> None:
        for e in self.get_sub_environments():
            if hasattr(e, "close"):
                e.close()

    @property
    def observation_space(self):
        raise NotImplementedError

    @property
    def action_space(self):
        raise NotImplementedError

    def to_base_env(self, *a, **k) -> "BaseEnv":
        return self


class _VectorBaseEnv(BaseEnv):
    """Sub-envs that are gym-style (single agent, id ``agent0``) or MultiAgentEnvs."""

    def __init__(self, envs: List[Any]):
        from ray_amd.rllib.env.multi_agent_env import MultiAgentEnv

        self.envs = list(envs)
        self.multi = [isinstance(e, MultiAgentEnv) for e in self.envs]
        self._pending: Dict[int, tuple] = {}
        for i in range(len(self.envs)):
            self._reset(i)

    def _reset(self, i, seed=None, options=None):
        obs, info = self.envs[i].reset(seed=seed, options=options)
        if not self.multi[i]:
            obs, info = {_DUMMY_AGENT_ID: obs}, {_DUMMY_AGENT_ID: info}
        self._pending[i] = (obs, {}, {"__all__": False}, {"__all__": False}, info)
        return obs, info

    def poll(self):
        o, r, te, tr, inf, off = {}, {}, {}, {}, {}, {}
        for i, (obs, rew, term, trunc, info) in self._pending.items():
            o[i], r[i], te[i], tr[i], inf[i], off[i] = obs, rew, term, trunc, info, {}
        self._pending = {}
        return o, r, te, tr, inf, off

    def send_actions(self, action_dict):
        for i, acts in action_dict.items():
            e = self.envs[i]
            if self.multi[i]:
                obs, rew, term, trunc, info = e.step(acts)
            else:
                ob, rw, t, u, inf = e.step(acts[_DUMMY_AGENT_ID])
                obs, rew, info = {_DUMMY_AGENT_ID: ob}, {_DUMMY_AGENT_ID: rw}, \
                    {_DUMMY_AGENT_ID: inf}
                term = {_DUMMY_AGENT_ID: t, "__all__": t}
                trunc = {_DUMMY_AGENT_ID: u, "__all__": u}
            self._pending[i] = (obs, rew, term, trunc, info)

    def try_reset(self, env_id=None, *, seed=None, options=None):
        ids = range(len(self.envs)) if env_id is None else [env_id]
        out_o, out_i = {}, {}
        for i in ids:
            out_o[i], out_i[i] = self._reset(i, seed, options)
        return out_o, out_i

    def get_sub_environments(self, as_dict: bool = False):
        return dict(enumerate(self.envs)) if as_dict else list(self.envs)

    def get_agent_ids(self):
        e = self.envs[0]
        return e.get_agent_ids() if self.multi[0] else {_DUMMY_AGENT_ID}

    @property
    def observation_space(self):
        return self.envs[0].observation_space

    @property
    def action_space(self):
        return self.envs[0].action_space


def convert_to_base_env(env, make_env=None, num_envs: int = 1,
                        remote_envs: bool = False, **kwargs) -> BaseEnv:
    """``env`` as a BaseEnv: a BaseEnv as is; a VectorEnv by its sub-environments; a
    gym-style or multi-agent env plus ``num_envs - 1`` more from ``make_env(i)``."""
    if remote_envs:
        raise NotImplementedError("remote_worker_envs: run more env runners instead")
    if isinstance(env, BaseEnv):
        return env
    from ray_amd.rllib.env.external_env import ExternalEnv, ExternalEnvAdapter
    from ray_amd.rllib.env.vector_env import VectorEnv

    if isinstance(env, VectorEnv):
        return _VectorBaseEnv(env.get_sub_environments())
    if isinstance(env, ExternalEnv):
        env = ExternalEnvAdapter(env)
    envs = [env] + [make_env(i) for i in range(1, num_envs)] if make_env else [env]
    return _VectorBaseEnv(envs)


class RemoteBaseEnv(BaseEnv):
    """The reference's BaseEnv over remote env actors (``remote_worker_envs``); ray_amd
    scales env stepping with more EnvRunners instead."""

    def __init__(self, *a, **k):
        raise NotImplementedError("remote_worker_envs is not supported: use more "
                                  "EnvRunners (num_env_runners / num_envs_per_env_runner)")


class ExternalMultiAgentEnv:
    """The reference's multi-agent ExternalEnv; ray_amd's ExternalEnv adapter is
    single-agent."""

    def __init__(self, *a, **k):
        raise NotImplementedError("ExternalMultiAgentEnv is not supported: use ExternalEnv "
                                  "(single agent) or a MultiAgentEnv")
