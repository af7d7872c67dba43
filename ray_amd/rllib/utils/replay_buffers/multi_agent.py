"""Multi-agent and FIFO replay buffers (reference: python/ray/rllib/utils/replay_buffers/
{multi_agent_replay_buffer,multi_agent_prioritized_replay_buffer,
multi_agent_mixin_replay_buffer,fifo_replay_buffer,utils}.py).

A multi-agent buffer keeps one column-store buffer (``ReplayBuffer`` /
``PrioritizedReplayBuffer``) per policy id; ``add`` takes a ``MultiAgentBatch`` or
``{policy_id: batch}``, ``sample(n)`` returns ``{policy_id: batch}`` with ``n`` items per
policy. ``ReplayMode.LOCKSTEP`` stores the policies' columns side by side in one buffer
(sampling the same rows for all)."""

from __future__ import annotations

from enum import Enum
from typing import Any, Dict, Optional

import numpy as np

from ray_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer

DEFAULT_POLICY_ID = "default_policy"


class ReplayMode(str, Enum):
    LOCKSTEP = "lockstep"
    INDEPENDENT = "independent"


class StorageUnit(str, Enum):
    TIMESTEPS = "timesteps"
    SEQUENCES = "sequences"
    EPISODES = "episodes"
    FRAGMENTS = "fragments"


def _policy_batches(batch) -> Dict[Any, dict]:
    pb = getattr(batch, "policy_batches", None)
    if pb is not None:
        return {k: dict(v) for k, v in pb.items()}
    if isinstance(batch, dict) and batch and all(isinstance(v, dict) for v in batch.values()):
        return {k: dict(v) for k, v in batch.items()}
    return {DEFAULT_POLICY_ID: dict(batch)}


class MultiAgentReplayBuffer:
    _underlying = ReplayBuffer

    def __init__(self, capacity: int = 10000, storage_unit: str = StorageUnit.TIMESTEPS,
                 replay_mode: str = ReplayMode.INDEPENDENT, seed=None,
                 underlying_buffer_config: Optional[dict] = None, **kwargs):
        self.capacity = int(capacity)
        self.storage_unit = StorageUnit(storage_unit)
        if self.storage_unit != StorageUnit.TIMESTEPS:
            raise NotImplementedError("multi-agent buffers store timesteps here; use "
                                      "EpisodeReplayBuffer for episodes")
        self.replay_mode = ReplayMode(replay_mode)
        self._seed = seed
        self._kw = dict(underlying_buffer_config or {})
        self._kw.pop("type", None)
        self._kw.update({k: v for k, v in kwargs.items() if k in ("alpha",)})
        self.replay_buffers: Dict[Any, ReplayBuffer] = {}
        self._num_added = 0

    def _buffer(self, pid) -> ReplayBuffer:
        if pid not in self.replay_buffers:
            self.replay_buffers[pid] = self._underlying(self.capacity, seed=self._seed,
                                                        **self._kw)
        return self.replay_buffers[pid]

    def __len__(self):
        return sum(len(b) for b in self.replay_buffers.values())

    def add(self, batch, **kwargs) -> None:
        pbs = _policy_batches(batch)
        if self.replay_mode == ReplayMode.LOCKSTEP:
            joined = {f"{pid}/{k}": v for pid, b in pbs.items() for k, v in b.items()}
            self._buffer("__all__").add(joined)
        else:
            for pid, b in pbs.items():
                self._buffer(pid).add(b, **kwargs) if kwargs else self._buffer(pid).add(b)
        self._num_added += max(len(next(iter(b.values()))) for b in pbs.values())

    def sample(self, num_items: int, policy_id=None, **kwargs) -> Dict[Any, dict]:
        if self.replay_mode == ReplayMode.LOCKSTEP:
            flat = self._buffer("__all__").sample(num_items, **kwargs)
            out: Dict[Any, dict] = {}
            for k, v in flat.items():
                if "/" in k:
                    pid, col = k.split("/", 1)
                    out.setdefault(pid, {})[col] = v
            return out
        pids = [policy_id] if policy_id is not None else list(self.replay_buffers)
        return {pid: self.replay_buffers[pid].sample(num_items, **kwargs) for pid in pids
                if pid in self.replay_buffers and len(self.replay_buffers[pid])}

    def stats(self, debug: bool = False) -> dict:
        return {"added_count": self._num_added,
                **{f"policy_{pid}": b.stats() for pid, b in self.replay_buffers.items()}}

    def get_state(self) -> dict:
        return {"added": self._num_added,
                "buffers": {pid: b.get_state() for pid, b in self.replay_buffers.items()}}

    def set_state(self, state: dict) -> None:
        self._num_added = state["added"]
        for pid, s in state["buffers"].items():
            self._buffer(pid).set_state(s)


class MultiAgentPrioritizedReplayBuffer(MultiAgentReplayBuffer):
    _underlying = PrioritizedReplayBuffer

    def __init__(self, capacity: int = 10000, prioritized_replay_alpha: float = 0.6,
                 prioritized_replay_beta: float = 0.4, **kwargs):
        kwargs.setdefault("underlying_buffer_config", {})["alpha"] = prioritized_replay_alpha
        super().__init__(capacity, **kwargs)
        self.beta = prioritized_replay_beta

    def sample(self, num_items: int, policy_id=None, beta: Optional[float] = None, **kw):
        return super().sample(num_items, policy_id, beta=self.beta if beta is None else beta)

    def update_priorities(self, prio_dict: Dict[Any, tuple]) -> None:
        """``{policy_id: (batch_indexes, td_errors)}``."""
        for pid, (idx, td) in prio_dict.items():
            self.replay_buffers[pid].update_priorities(idx, np.abs(np.asarray(td)))


class MultiAgentMixInReplayBuffer(MultiAgentReplayBuffer):
    """Mixes the newest added samples into every sampled batch: with
    ``replay_ratio`` r, a batch is (1 - r) new and r replayed (reference:
    multi_agent_mixin_replay_buffer.py)."""

    def __init__(self, capacity: int = 10000, replay_ratio: float = 0.66, **kwargs):
        super().__init__(capacity, **kwargs)
        if not 0.0 <= replay_ratio <= 1.0:
            raise ValueError("replay_ratio must be in [0, 1]")
        self.replay_ratio = replay_ratio
        self._last: Dict[Any, dict] = {}

    def add(self, batch, **kwargs) -> None:
        pbs = _policy_batches(batch)
        for pid, b in pbs.items():
            self._last[pid] = {k: np.asarray(v) for k, v in b.items()}
        super().add(batch, **kwargs)

    def sample(self, num_items: int, policy_id=None, **kwargs) -> Dict[Any, dict]:
        out = {}
        pids = [policy_id] if policy_id is not None else list(self.replay_buffers)
        for pid in pids:
            new = self._last.pop(pid, None)
            n_new = 0 if new is None else len(next(iter(new.values())))
            if self.replay_ratio >= 1.0 or n_new == 0:
                n_old = num_items
            elif self.replay_ratio == 0.0:
                n_old = 0
            else:
                n_old = int(round(n_new * self.replay_ratio / (1 - self.replay_ratio)))
            parts = [new] if n_new else []
            if n_old and len(self.replay_buffers.get(pid, ())):
                old = self.replay_buffers[pid].sample(n_old)
                old.pop("batch_indexes", None)
                parts.append(old)
            if parts:
                keys = set.intersection(*[set(p) for p in parts])
                out[pid] = {k: np.concatenate([np.asarray(p[k]) for p in parts]) for k in keys}
        return out


class FifoReplayBuffer(ReplayBuffer):
    """Returns the added items in insertion order, each once (a queue, for on-policy
    data flowing through the replay API)."""

    def __init__(self, capacity: int = 10000, seed=None, **kwargs):
        super().__init__(capacity, seed)
        self._read = 0

    def sample(self, num_items: Optional[int] = None, **kw) -> dict:
        avail = self._num_added - self._read
        if avail <= 0:
            return {}
        n = avail if num_items is None else min(num_items, avail)
        start = self._read
        idx = (np.arange(start, start + n)) % self.capacity
        self._read += n
        out = {k: v[idx] for k, v in self._cols.items()}
        out["batch_indexes"] = idx
        return out
