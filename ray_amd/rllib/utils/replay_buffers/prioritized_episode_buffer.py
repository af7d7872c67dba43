"""``PrioritizedEpisodeReplayBuffer`` (reference: python/ray/rllib/utils/replay_buffers/
prioritized_episode_buffer.py): an EpisodeReplayBuffer whose timesteps are sampled in
proportion to ``priority ** alpha`` with importance weights ``(N p)^-beta / max``. New
timesteps get the highest priority seen so far; ``update_priorities(td_errors)`` sets the
priorities of the last sampled batch's timesteps."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.utils.replay_buffers.episode_replay_buffer import EpisodeReplayBuffer


class PrioritizedEpisodeReplayBuffer(EpisodeReplayBuffer):
    def __init__(self, capacity: int = 10000, *, batch_size_B: int = 16,
                 batch_length_T: int = 1, alpha: float = 1.0, seed=None, **kwargs):
        super().__init__(capacity, batch_size_B=batch_size_B, batch_length_T=batch_length_T,
                         seed=seed, **kwargs)
        self._alpha = float(alpha)
        self._prio = {}  # episode id -> per-timestep priority (already ** alpha)
        self._max_priority = 1.0
        self._last = None  # (episode ids, timesteps) of the last sample

    def add(self, episodes, weight=None):
        from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode

        if isinstance(episodes, SingleAgentEpisode):
            episodes = [episodes]
        for ep in episodes:
            p = (self._max_priority if weight is None else float(weight)) ** self._alpha
            new = np.full(len(ep), p)
            self._prio[ep.id_] = np.concatenate([self._prio[ep.id_], new]) \
                if ep.id_ in self._prio else new
        super().add(episodes)
        for eid in list(self._prio):
            if eid not in self.episodes:
                del self._prio[eid]

    def sample(self, num_items=None, *, batch_size_B=None, batch_length_T=None, n_step=1,
               gamma=0.99, beta: float = 0.0, **kw):
        B = int(batch_size_B or num_items or self.batch_size_B)
        eps = [e for e in self.episodes.values() if len(e)]
        if not eps:
            raise ValueError("the buffer holds no timesteps")
        pr = np.concatenate([self._prio[e.id_][:len(e)] for e in eps])
        lens = np.array([len(e) for e in eps])
        cum = np.cumsum(lens)
        probs = pr / pr.sum()
        picks = self.rng.choice(len(pr), size=B, p=probs)
        which = np.searchsorted(cum, picks, side="right")
        ts = picks - (cum[which] - lens[which])
        obs, nobs, acts, rews, terms, disc = [], [], [], [], [], []
        n_step = max(1, int(n_step))
        for w, t in zip(which, ts):
            e = eps[w]
            t = int(t)
            k = min(n_step, len(e) - t)
            rews.append(sum((gamma ** j) * e.rewards[t + j] for j in range(k)))
            obs.append(e.observations[t])
            nobs.append(e.observations[t + k])
            acts.append(e.actions[t])
            terms.append(1.0 if (e.is_terminated and t + k == len(e)) else 0.0)
            disc.append(gamma ** k)
        N = len(pr)
        w = (N * probs[picks]) ** (-beta)
        w = w / ((N * probs.min()) ** (-beta))
        self._last = ([eps[i].id_ for i in which], ts.astype(np.int64))
        return {"obs": np.stack(obs), "next_obs": np.stack(nobs), "actions": np.asarray(acts),
                "rewards": np.asarray(rews, np.float32),
                "terminateds": np.asarray(terms, np.float32),
                "discounts": np.asarray(disc, np.float32), "weights": w.astype(np.float32),
                "n_step": np.full(B, n_step, np.int64)}

    def update_priorities(self, priorities, module_id=None) -> None:
        if self._last is None:
            raise ValueError("update_priorities needs a preceding sample()")
        ids, ts = self._last
        pr = np.abs(np.asarray(priorities, np.float64)) + 1e-6
        for eid, t, p in zip(ids, ts, pr):
            if eid in self._prio and t < len(self._prio[eid]):
                self._prio[eid][t] = p ** self._alpha
        self._max_priority = max(self._max_priority, float(pr.max()))

    def get_state(self):
        s = super().get_state()
        s["prio"] = {k: v.copy() for k, v in self._prio.items()}
        s["max_priority"] = self._max_priority
        return s

    def set_state(self, s):
        super().set_state(s)
        self._prio = {k: np.asarray(v) for k, v in s.get("prio", {}).items()}
        self._max_priority = s.get("max_priority", 1.0)
