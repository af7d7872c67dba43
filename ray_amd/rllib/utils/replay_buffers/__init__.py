"""Replay buffers (reference: rllib/utils/replay_buffers/{replay_buffer,
prioritized_replay_buffer,reservoir_replay_buffer}.py, rllib/execution/segment_tree.py).

Storage is a set of preallocated column arrays (ring buffer) rather than a list of
SampleBatch objects, so sampling a minibatch is one fancy-index gather per column
(ready for a single pinned H2D copy to the learner GPU)."""

from __future__ import annotations

import numpy as np


class ReplayBuffer:
    def __init__(self, capacity: int = 10000, seed=None):
        self.capacity = int(capacity)
        self._cols = None
        self._next = 0
        self._size = 0
        self._num_added = 0
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return self._size

    def _alloc(self, batch):
        self._cols = {}
        for k, v in batch.items():
            v = np.asarray(v)
            self._cols[k] = np.zeros((self.capacity,) + v.shape[1:], dtype=v.dtype)

    def add(self, batch: dict):
        """batch: dict of arrays with a leading item dimension."""
        n = len(next(iter(batch.values())))
        if self._cols is None:
            self._alloc(batch)
        idx = (self._next + np.arange(n)) % self.capacity
        for k, v in batch.items():
            self._cols[k][idx] = v
        self._next = int((self._next + n) % self.capacity)
        self._size = min(self.capacity, self._size + n)
        self._num_added += n
        return idx

    def sample(self, num_items: int, **kw) -> dict:
        if self._size == 0:
            raise ValueError("cannot sample from an empty buffer")
        idx = self.rng.integers(0, self._size, size=num_items)
        out = {k: v[idx] for k, v in self._cols.items()}
        out["batch_indexes"] = idx
        return out

    def stats(self):
        return {"added_count": self._num_added, "num_entries": self._size}

    def get_state(self):
        return {"cols": self._cols, "next": self._next, "size": self._size,
                "added": self._num_added}

    def set_state(self, s):
        self._cols, self._next, self._size, self._num_added = s["cols"], s["next"], s["size"], \
            s["added"]


class SumSegmentTree:
    """Array-backed sum tree with prefix-sum search (reference: execution/segment_tree.py)."""

    def __init__(self, capacity):
        c = 1
        while c < capacity:
            c *= 2
        self.capacity = c
        self.value = np.zeros(2 * c, dtype=np.float64)

    def __setitem__(self, idx, val):
        idx = np.atleast_1d(np.asarray(idx)) + self.capacity
        val = np.broadcast_to(np.asarray(val, dtype=np.float64), idx.shape)
        for i, v in zip(idx, val):
            self.value[i] = v
            i //= 2
            while i >= 1:
                self.value[i] = self.value[2 * i] + self.value[2 * i + 1]
                i //= 2

    def __getitem__(self, idx):
        return self.value[np.asarray(idx) + self.capacity]

    def sum(self):
        return self.value[1]

    def find_prefixsum_idx(self, prefixsum):
        out = np.empty(len(prefixsum), dtype=np.int64)
        for j, p in enumerate(prefixsum):
            i = 1
            while i < self.capacity:
                if self.value[2 * i] > p:
                    i = 2 * i
                else:
                    p -= self.value[2 * i]
                    i = 2 * i + 1
            out[j] = i - self.capacity
        return out


class MinSegmentTree:
    def __init__(self, capacity):
        c = 1
        while c < capacity:
            c *= 2
        self.capacity = c
        self.value = np.full(2 * c, np.inf)

    def __setitem__(self, idx, val):
        idx = np.atleast_1d(np.asarray(idx)) + self.capacity
        val = np.broadcast_to(np.asarray(val, dtype=np.float64), idx.shape)
        for i, v in zip(idx, val):
            self.value[i] = v
            i //= 2
            while i >= 1:
                self.value[i] = min(self.value[2 * i], self.value[2 * i + 1])
                i //= 2

    def min(self):
        return self.value[1]


class PrioritizedReplayBuffer(ReplayBuffer):
    """Proportional prioritized replay (Schaul et al. 2016)."""

    def __init__(self, capacity: int = 10000, alpha: float = 0.6, seed=None):
        super().__init__(capacity, seed)
        self.alpha = alpha
        self._sum = SumSegmentTree(self.capacity)
        self._min = MinSegmentTree(self.capacity)
        self._max_priority = 1.0

    def add(self, batch, weight=None):
        idx = super().add(batch)
        p = (self._max_priority if weight is None else weight) ** self.alpha
        self._sum[idx] = p
        self._min[idx] = p
        return idx

    def sample(self, num_items: int, beta: float = 0.4, **kw):
        total = self._sum.sum()
        mass = (self.rng.random(num_items) + np.arange(num_items)) * (total / num_items)
        idx = np.minimum(self._sum.find_prefixsum_idx(mass), self._size - 1)
        p_min = self._min.min() / total
        max_w = (p_min * self._size) ** (-beta)
        p = self._sum[idx] / total
        w = (p * self._size) ** (-beta) / max_w
        out = {k: v[idx] for k, v in self._cols.items()}
        out["weights"] = w.astype(np.float32)
        out["batch_indexes"] = idx
        return out

    def update_priorities(self, idxes, priorities):
        priorities = np.asarray(priorities, dtype=np.float64) + 1e-6
        self._sum[idxes] = priorities ** self.alpha
        self._min[idxes] = priorities ** self.alpha
        self._max_priority = max(self._max_priority, float(priorities.max()))


class ReservoirReplayBuffer(ReplayBuffer):
    """Reservoir sampling: every item ever added has equal probability to be stored."""

    def add(self, batch):
        n = len(next(iter(batch.values())))
        if self._cols is None:
            self._alloc(batch)
        for j in range(n):
            self._num_added += 1
            if self._size < self.capacity:
                i = self._size
                self._size += 1
            else:
                i = int(self.rng.integers(0, self._num_added))
                if i >= self.capacity:
                    continue
            for k, v in batch.items():
                self._cols[k][i] = v[j]


from ray_amd.rllib.utils.replay_buffers.episode_replay_buffer import (  # noqa: E402,F401
    EpisodeReplayBuffer)
from ray_amd.rllib.utils.replay_buffers.multi_agent import (  # noqa: E402,F401
    FifoReplayBuffer, MultiAgentMixInReplayBuffer, MultiAgentPrioritizedReplayBuffer,
    MultiAgentReplayBuffer, ReplayMode, StorageUnit)
from ray_amd.rllib.utils.replay_buffers.prioritized_episode_buffer import (  # noqa: E402,F401
    PrioritizedEpisodeReplayBuffer)
from ray_amd.rllib.utils.replay_buffers import utils  # noqa: E402,F401
