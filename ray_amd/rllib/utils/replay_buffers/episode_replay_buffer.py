"""EpisodeReplayBuffer (reference: rllib/utils/replay_buffers/episode_replay_buffer.py:14).

Stores whole episodes (chunks of an ongoing episode are concatenated by id) up to
``capacity`` env steps, evicting the oldest episodes first, and samples uniformly over all
stored timesteps. ``sample(batch_size_B, n_step=k, gamma=g)`` returns n-step transitions:
the discounted reward sum over up to k steps (cut at the episode end), the observation k'
steps later, ``terminateds`` when that window reaches a terminal step and the per-row
bootstrap discount ``gamma ** k'`` (column ``discounts``)."""

from __future__ import annotations

import collections

import numpy as np

from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode


class EpisodeReplayBuffer:
    def __init__(self, capacity: int = 10000, *, batch_size_B: int = 16,
                 batch_length_T: int = 1, seed=None, **kwargs):
        self.capacity = int(capacity)
        self.batch_size_B = batch_size_B
        self.batch_length_T = batch_length_T
        self.episodes = collections.OrderedDict()  # id -> SingleAgentEpisode
        self._num_timesteps = 0
        self._num_timesteps_added = 0
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return self._num_timesteps

    def get_num_timesteps(self):
        return self._num_timesteps

    def get_num_episodes(self):
        return len(self.episodes)

    def get_added_timesteps(self):
        return self._num_timesteps_added

    def add(self, episodes):
        if isinstance(episodes, SingleAgentEpisode):
            episodes = [episodes]
        for ep in episodes:
            n = len(ep)
            if ep.id_ in self.episodes:
                self.episodes[ep.id_].concat_episode(ep)
            else:
                self.episodes[ep.id_] = SingleAgentEpisode.from_state(ep.get_state())
            self._num_timesteps += n
            self._num_timesteps_added += n
        while self._num_timesteps > self.capacity and len(self.episodes) > 1:
            _, old = self.episodes.popitem(last=False)
            self._num_timesteps -= len(old)

    def sample(self, num_items=None, *, batch_size_B=None, batch_length_T=None, n_step=1,
               gamma=0.99, **kw):
        """Uniform over timesteps; returns a dict of numpy columns."""
        B = int(batch_size_B or num_items or self.batch_size_B)
        eps = [e for e in self.episodes.values() if len(e)]
        if not eps:
            raise ValueError("the buffer holds no timesteps")
        lens = np.array([len(e) for e in eps])
        cum = np.cumsum(lens)
        picks = self.rng.integers(0, int(cum[-1]), size=B)
        which = np.searchsorted(cum, picks, side="right")
        obs, nobs, acts, rews, terms, disc = [], [], [], [], [], []
        n_step = max(1, int(n_step))
        for w, p in zip(which, picks):
            e = eps[w]
            t = int(p - (cum[w] - lens[w]))
            k = min(n_step, len(e) - t)
            r = 0.0
            for j in range(k):
                r += (gamma ** j) * e.rewards[t + j]
            obs.append(e.observations[t])
            nobs.append(e.observations[t + k])
            acts.append(e.actions[t])
            rews.append(r)
            terms.append(1.0 if (e.is_terminated and t + k == len(e)) else 0.0)
            disc.append(gamma ** k)
        return {"obs": np.stack(obs), "next_obs": np.stack(nobs), "actions": np.asarray(acts),
                "rewards": np.asarray(rews, np.float32),
                "terminateds": np.asarray(terms, np.float32),
                "discounts": np.asarray(disc, np.float32),
                "weights": np.ones(B, np.float32)}

    def get_state(self):
        return {"episodes": [e.get_state() for e in self.episodes.values()],
                "added": self._num_timesteps_added}

    def set_state(self, s):
        self.episodes.clear()
        self._num_timesteps = 0
        for st in s["episodes"]:
            e = SingleAgentEpisode.from_state(st)
            self.episodes[e.id_] = e
            self._num_timesteps += len(e)
        self._num_timesteps_added = s.get("added", self._num_timesteps)
