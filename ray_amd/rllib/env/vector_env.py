"""Vectorised environments (reference: rllib/env/vector_env.py).

``VectorEnv`` is the batched-env interface (``vector_reset`` / ``vector_step`` over
``num_envs`` sub-environments, ``reset_at`` for one index). ``VectorEnv.vectorize_gym_envs``
builds one from an env factory or existing envs, optionally recreating sub-environments
whose ``step`` raises (``restart_failed_sub_environments``: the failed slot reports a
truncated episode with ``info["env_error"]`` and is rebuilt on the next reset).

EnvRunners already step ``num_envs_per_env_runner`` envs in lock-step; an env creator
that returns a VectorEnv with concrete sub-environments contributes all of them to the
runner (``SingleAgentEnvRunner`` flattens ``get_sub_environments()``).
"""

from __future__ import annotations

import logging

logger = logging.getLogger(__name__)


class VectorEnv:
    def __init__(self, observation_space, action_space, num_envs: int):
        self.observation_space = observation_space
        self.action_space = action_space
        self.num_envs = num_envs

    @staticmethod
    def vectorize_gym_envs(make_env=None, existing_envs=None, num_envs: int = 1,
                           action_space=None, observation_space=None,
                           restart_failed_sub_environments: bool = False,
                           env_config=None) -> "_VectorizedEnvs":
        return _VectorizedEnvs(make_env, list(existing_envs or []), num_envs,
                               observation_space, action_space,
                               restart_failed_sub_environments, env_config)

    def vector_reset(self, *, seeds=None, options=None):
        raise NotImplementedError

    def reset_at(self, index: int | None = None, *, seed=None, options=None):
        raise NotImplementedError

    def restart_at(self, index: int | None = None) -> None:
        raise NotImplementedError

    def vector_step(self, actions):
        raise NotImplementedError

    def get_sub_environments(self) -> list:
        return []

    def try_render_at(self, index: int | None = None):
        return None

    def close(self):
        for e in self.get_sub_environments():
            try:
                e.close()
            except Exception:  # noqa: BLE001
                pass


class _VectorizedEnvs(VectorEnv):
    def __init__(self, make_env, existing, num_envs, obs_space, act_space, restart, env_config):
        self.make_env = make_env
        self.restart_failed = restart
        self.env_config = env_config or {}
        self.envs = existing
        while len(self.envs) < num_envs:
            if make_env is None:
                raise ValueError("vectorize_gym_envs needs make_env to create "
                                 f"{num_envs - len(self.envs)} more sub-environments")
            self.envs.append(self._make(len(self.envs)))
        self._failed = [False] * len(self.envs)
        super().__init__(obs_space or self.envs[0].observation_space,
                         act_space or self.envs[0].action_space, len(self.envs))

    def _make(self, i):
        try:
            return self.make_env(i)
        except TypeError:
            return self.make_env()

    def vector_reset(self, *, seeds=None, options=None):
        seeds = seeds if seeds is not None else [None] * self.num_envs
        options = options if options is not None else [None] * self.num_envs
        obs, infos = [], []
        for i in range(self.num_envs):
            o, inf = self.reset_at(i, seed=seeds[i], options=options[i])
            obs.append(o)
            infos.append(inf)
        return obs, infos

    def reset_at(self, index=None, *, seed=None, options=None):
        i = 0 if index is None else index
        if self._failed[i]:
            self.restart_at(i)
        return self.envs[i].reset(seed=seed, options=options)

    def restart_at(self, index=None):
        i = 0 if index is None else index
        try:
            self.envs[i].close()
        except Exception:  # noqa: BLE001 - the env already failed
            pass
        self.envs[i] = self._make(i)
        self._failed[i] = False

    def vector_step(self, actions):
        obs, rews, terms, truncs, infos = [], [], [], [], []
        for i, a in enumerate(actions):
            try:
                o, r, te, tr, inf = self.envs[i].step(a)
            except Exception as e:  # noqa: BLE001
                if not self.restart_failed:
                    raise
                logger.warning("sub-environment %d failed (%r); it is restarted", i, e)
                self._failed[i] = True
                o, r, te, tr, inf = (self.observation_space.sample(), 0.0, False, True,
                                     {"env_error": repr(e)})
            obs.append(o)
            rews.append(r)
            terms.append(te)
            truncs.append(tr)
            infos.append(inf)
        return obs, rews, terms, truncs, infos

    def get_sub_environments(self):
        return self.envs

    def try_render_at(self, index=None):
        return self.envs[0 if index is None else index].render()


__all__ = ["VectorEnv"]
