"""Old-stack batch builders (reference: python/ray/rllib/evaluation/sample_batch_builder.py):
append rows one at a time, ``build_and_reset()`` returns a SampleBatch (or a
MultiAgentBatch with one SampleBatch per policy)."""

from __future__ import annotations

import collections
from typing import Any, Dict

import numpy as np

from ray_amd.rllib.policy_sample_batch import MultiAgentBatch, SampleBatch


class SampleBatchBuilder:
    def __init__(self):
        self.buffers: Dict[str, list] = collections.defaultdict(list)
        self.count = 0

    def add_values(self, **values: Any) -> None:
        for k, v in values.items():
            self.buffers[k].append(v)
        self.count += 1

    def add_batch(self, batch) -> None:
        for k, v in dict(batch).items():
            self.buffers[k].extend(list(v))
        self.count += len(next(iter(dict(batch).values()))) if len(batch) else 0

    def build_and_reset(self) -> SampleBatch:
        out = SampleBatch({k: np.asarray(v) for k, v in self.buffers.items()})
        self.buffers.clear()
        self.count = 0
        return out


class MultiAgentSampleBatchBuilder:
    def __init__(self, policy_map=None, clip_rewards: bool = False, callbacks=None):
        self.policy_builders: Dict[Any, SampleBatchBuilder] = collections.defaultdict(
            SampleBatchBuilder)
        self.clip_rewards = clip_rewards
        self.count = 0

    def add_values(self, agent_id, policy_id, **values: Any) -> None:
        if self.clip_rewards and "rewards" in values:
            values["rewards"] = float(np.sign(values["rewards"]))
        self.policy_builders[policy_id].add_values(agent_id=agent_id, **values)

    def total(self) -> int:
        return sum(b.count for b in self.policy_builders.values())

    def has_pending_agent_data(self) -> bool:
        return self.total() > 0

    def build_and_reset(self, episode=None) -> MultiAgentBatch:
        batches = {pid: b.build_and_reset() for pid, b in self.policy_builders.items()
                   if b.count}
        self.policy_builders.clear()
        env_steps = self.count or max((len(b) for b in batches.values()), default=0)
        self.count = 0
        return MultiAgentBatch(batches, env_steps)
