"""SingleAgentEpisode (reference: rllib/env/single_agent_episode.py:18).

One (chunk of an) episode of a single agent: ``len(observations) == len(actions) + 1``
(the episode's reset observation comes first). An ongoing episode is ``cut()`` at the end
of a rollout; the successor chunk keeps the episode id and starts at the last observation,
and ``concat_episode`` glues chunks back together (the episode replay buffer does that)."""

from __future__ import annotations

import uuid

import numpy as np


class SingleAgentEpisode:
    def __init__(self, id_=None, *, observations=None, actions=None, rewards=None,
                 infos=None, terminated=False, truncated=False, extra_model_outputs=None,
                 t_started=0, len_lookback_buffer=0, observation_space=None,
                 action_space=None):
        self.id_ = id_ or uuid.uuid4().hex
        self.observations = list(observations or [])
        self.actions = list(actions or [])
        self.rewards = list(rewards or [])
        self.infos = list(infos or [{} for _ in self.observations])
        self.extra_model_outputs = {k: list(v) for k, v in (extra_model_outputs or {}).items()}
        self.is_terminated = bool(terminated)
        self.is_truncated = bool(truncated)
        self.t_started = t_started
        self.t = t_started + len(self.actions)
        self.observation_space = observation_space
        self.action_space = action_space
        self._finalized = False

    # ---------------------------------------------------------------- building
    def add_env_reset(self, observation, infos=None):
        if self.observations:
            raise ValueError("add_env_reset() on an episode that already has observations")
        self.observations.append(observation)
        self.infos.append(infos or {})

    def add_env_step(self, observation, action, reward, infos=None, *, terminated=False,
                     truncated=False, extra_model_outputs=None):
        if self.is_done:
            raise ValueError(f"episode {self.id_} is already done")
        if not self.observations:
            raise ValueError("add_env_step() before add_env_reset()")
        self.observations.append(observation)
        self.actions.append(action)
        self.rewards.append(float(reward))
        self.infos.append(infos or {})
        for k, v in (extra_model_outputs or {}).items():
            self.extra_model_outputs.setdefault(k, []).append(v)
        self.is_terminated = bool(terminated)
        self.is_truncated = bool(truncated)
        self.t += 1

    @property
    def is_done(self) -> bool:
        return self.is_terminated or self.is_truncated

    def __len__(self) -> int:
        return len(self.actions)

    def env_steps(self) -> int:
        """Env steps in this chunk (reference: SingleAgentEpisode.env_steps)."""
        return len(self)

    def agent_steps(self) -> int:
        """Same as ``env_steps`` for a single agent."""
        return len(self)

    @property
    def is_finalized(self) -> bool:
        return self._finalized

    def validate(self) -> None:
        """The chunk invariants: one more observation / info than actions, rewards and
        each extra-model-output column."""
        n = len(self.actions)
        if len(self.observations) != n + 1 and not (n == 0 and len(self.observations) <= 1):
            raise AssertionError(f"{len(self.observations)} observations for {n} actions")
        if len(self.rewards) != n:
            raise AssertionError(f"{len(self.rewards)} rewards for {n} actions")
        if len(self.infos) != len(self.observations):
            raise AssertionError(f"{len(self.infos)} infos for {len(self.observations)} obs")
        for k, v in self.extra_model_outputs.items():
            if len(v) != n:
                raise AssertionError(f"extra_model_outputs[{k!r}] has {len(v)} rows for {n}")

    def get_return(self) -> float:
        return float(np.sum(self.rewards)) if self.rewards else 0.0

    def get_duration_s(self):
        return None

    # ---------------------------------------------------------------- access
    @staticmethod
    def _pick(lst, indices):
        if indices is None:
            return lst
        if isinstance(indices, slice):
            return lst[indices]
        if isinstance(indices, (list, tuple, np.ndarray)):
            return [lst[i] for i in indices]
        return lst[indices]

    def get_observations(self, indices=None):
        return self._pick(self.observations, indices)

    def get_actions(self, indices=None):
        return self._pick(self.actions, indices)

    def get_rewards(self, indices=None):
        return self._pick(self.rewards, indices)

    def get_infos(self, indices=None):
        return self._pick(self.infos, indices)

    def get_extra_model_outputs(self, key, indices=None):
        return self._pick(self.extra_model_outputs[key], indices)

    # ---------------------------------------------------------------- overwrite
    def _set(self, lst, new_data, at_indices):
        """Overwrite ``lst[at_indices]`` (an int, a slice, a list, or None = every row)."""
        if self._finalized:
            raise ValueError("set_*() on a finalized episode (numpy arrays): set before "
                             "finalize()")
        if isinstance(at_indices, int):
            lst[at_indices] = new_data
            return
        idx = list(range(len(lst))[at_indices]) if isinstance(at_indices, slice) else \
            list(range(len(lst))) if at_indices is None else list(at_indices)
        vals = list(new_data)
        if len(vals) != len(idx):
            raise IndexError(f"{len(vals)} values for {len(idx)} indices")
        for i, v in zip(idx, vals):
            lst[i] = v

    def set_observations(self, *, new_data, at_indices=None):
        self._set(self.observations, new_data, at_indices)

    def set_actions(self, *, new_data, at_indices=None):
        self._set(self.actions, new_data, at_indices)

    def set_rewards(self, *, new_data, at_indices=None):
        self._set(self.rewards, float(new_data) if isinstance(at_indices, int) else
                  [float(r) for r in np.atleast_1d(new_data)], at_indices)

    def set_extra_model_outputs(self, *, key, new_data, at_indices=None):
        col = self.extra_model_outputs.setdefault(key, [None] * len(self.actions))
        self._set(col, new_data, at_indices)

    # ---------------------------------------------------------------- batches
    def get_data_dict(self) -> dict:
        """Column dict of this chunk, one row per action: obs / next_obs, actions, rewards,
        terminateds / truncateds (last row only), t, eps_id and the extra model outputs."""
        n = len(self.actions)
        obs = np.asarray(self.observations)
        d = {"obs": obs[:n], "new_obs": obs[1:n + 1], "actions": np.asarray(self.actions),
             "rewards": np.asarray(self.rewards, np.float32),
             "terminateds": np.zeros(n, bool), "truncateds": np.zeros(n, bool),
             "t": np.arange(self.t_started, self.t_started + n),
             "eps_id": np.array([self.id_] * n)}
        if n:
            d["terminateds"][-1] = self.is_terminated
            d["truncateds"][-1] = self.is_truncated
        for k, v in self.extra_model_outputs.items():
            d[k] = np.asarray(v)
        return d

    def get_sample_batch(self):
        """The chunk as an old-stack ``SampleBatch``."""
        from ray_amd.rllib.policy_sample_batch import SampleBatch

        return SampleBatch(self.get_data_dict())

    # ---------------------------------------------------------------- chunks
    def cut(self, len_lookback_buffer=0) -> "SingleAgentEpisode":
        """The successor chunk of this (ongoing) episode: same id, starting at the last
        observation (reference: SingleAgentEpisode.cut)."""
        if self.is_done:
            raise ValueError("cannot cut a finished episode")
        return SingleAgentEpisode(self.id_, observations=[self.observations[-1]],
                                  infos=[self.infos[-1]], t_started=self.t,
                                  observation_space=self.observation_space,
                                  action_space=self.action_space)

    def concat_episode(self, other: "SingleAgentEpisode"):
        """Append the successor chunk ``other`` (its first observation must be this
        chunk's last)."""
        if other.id_ != self.id_:
            raise ValueError("can only concat chunks of the same episode")
        if self.is_done:
            raise ValueError("cannot extend a finished episode")
        if other.t_started != self.t:
            raise ValueError(f"chunk starts at t={other.t_started}, episode is at t={self.t}")
        self.observations.extend(other.observations[1:])
        self.infos.extend(other.infos[1:])
        self.actions.extend(other.actions)
        self.rewards.extend(other.rewards)
        for k, v in other.extra_model_outputs.items():
            self.extra_model_outputs.setdefault(k, []).extend(v)
        self.is_terminated, self.is_truncated = other.is_terminated, other.is_truncated
        self.t = other.t

    def slice(self, s: slice) -> "SingleAgentEpisode":
        start, stop, _ = s.indices(len(self))
        done = stop == len(self)
        return SingleAgentEpisode(
            self.id_, observations=self.observations[start:stop + 1],
            actions=self.actions[start:stop], rewards=self.rewards[start:stop],
            infos=self.infos[start:stop + 1],
            extra_model_outputs={k: v[start:stop] for k, v in self.extra_model_outputs.items()},
            terminated=self.is_terminated and done, truncated=self.is_truncated and done,
            t_started=self.t_started + start)

    def __getitem__(self, s):
        if not isinstance(s, slice):
            raise TypeError("episode indexing takes a slice")
        return self.slice(s)

    def finalize(self):
        """Lists -> numpy arrays (reference: episode.finalize / to_numpy)."""
        if not self._finalized:
            self.observations = np.asarray(self.observations)
            self.actions = np.asarray(self.actions)
            self.rewards = np.asarray(self.rewards, np.float32)
            self.extra_model_outputs = {k: np.asarray(v)
                                        for k, v in self.extra_model_outputs.items()}
            self._finalized = True
        return self

    to_numpy = finalize

    def get_state(self) -> dict:
        return {"id_": self.id_, "observations": list(self.observations),
                "actions": list(self.actions), "rewards": list(self.rewards),
                "infos": list(self.infos), "terminated": self.is_terminated,
                "truncated": self.is_truncated, "t_started": self.t_started,
                "extra_model_outputs": {k: list(v) for k, v in
                                        self.extra_model_outputs.items()}}

    @staticmethod
    def from_state(state) -> "SingleAgentEpisode":
        s = dict(state)
        return SingleAgentEpisode(s.pop("id_"), **s)

    def __repr__(self):
        return (f"SAEps(len={len(self)} done={self.is_done} R={self.get_return():.2f} "
                f"id_={self.id_})")
