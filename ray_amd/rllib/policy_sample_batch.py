"""``SampleBatch`` / ``MultiAgentBatch``: the columnar trajectory containers of RLlib's
classic API (reference: rllib/policy/sample_batch.py).

A SampleBatch is a dict of equal-length numpy columns (obs, actions, rewards, terminateds,
truncateds, eps_id, ...). Provided: column constants, ``concat_samples``, slicing and
``rows()``, ``shuffle``, ``split_by_episode``, ``timeslices``, ``right_zero_pad``,
``to_device`` (torch tensors, e.g. onto the learner's MI355X), ``get_single_step_input_dict``
is not needed by this stack. The env runners here emit column dicts of this exact shape,
so ``SampleBatch(runner_output)`` wraps them without copying.
"""

from __future__ import annotations

from typing import Dict, Iterable, List

import numpy as np


class SampleBatch(dict):
    OBS = "obs"
    NEXT_OBS = "new_obs"
    ACTIONS = "actions"
    REWARDS = "rewards"
    PREV_ACTIONS = "prev_actions"
    PREV_REWARDS = "prev_rewards"
    TERMINATEDS = "terminateds"
    TRUNCATEDS = "truncateds"
    INFOS = "infos"
    SEQ_LENS = "seq_lens"
    T = "t"
    EPS_ID = "eps_id"
    ENV_ID = "env_id"
    AGENT_INDEX = "agent_index"
    UNROLL_ID = "unroll_id"
    ACTION_DIST_INPUTS = "action_dist_inputs"
    ACTION_PROB = "action_prob"
    ACTION_LOGP = "action_logp"
    VF_PREDS = "vf_preds"
    VALUES_BOOTSTRAPPED = "values_bootstrapped"
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            if isinstance(v, list):
                self[k] = np.asarray(v)
        lens = {len(v) for k, v in self.items() if k != self.SEQ_LENS and hasattr(v, "__len__")}
        if len(lens) > 1:
            raise ValueError(f"SampleBatch columns have different lengths: {lens}")
        self.count = lens.pop() if lens else 0

    # --------------------------------------------------------------- size / access
    def __len__(self):
        return self.count

    @property
    def env_steps(self) -> int:
        return self.count

    def agent_steps(self) -> int:
        return self.count

    def rows(self) -> Iterable[Dict]:
        for i in range(self.count):
            yield {k: v[i] for k, v in self.items() if k != self.SEQ_LENS}

    def columns(self, keys: List[str]) -> List[np.ndarray]:
        return [self[k] for k in keys]

    def slice(self, start: int, end: int) -> "SampleBatch":
        return SampleBatch({k: v[start:end] for k, v in self.items() if k != self.SEQ_LENS})

    def __getitem__(self, key):
        if isinstance(key, slice):
            return self.slice(key.start or 0, self.count if key.stop is None else key.stop)
        return super().__getitem__(key)

    def copy(self, shallow: bool = False) -> "SampleBatch":
        return SampleBatch({k: (v if shallow else np.array(v, copy=True))
                            for k, v in self.items()})

    # --------------------------------------------------------------- transforms
    def concat(self, other: "SampleBatch") -> "SampleBatch":
        return concat_samples([self, other])

    def shuffle(self, seed=None) -> "SampleBatch":
        perm = np.random.default_rng(seed).permutation(self.count)
        for k in list(self):
            if k != self.SEQ_LENS:
                self[k] = np.asarray(self[k])[perm]
        return self

    def split_by_episode(self, key: str | None = None) -> List["SampleBatch"]:
        """Contiguous runs of one ``eps_id``; without eps_id, cut after every
        terminated/truncated step."""
        if key is None and self.EPS_ID in self:
            key = self.EPS_ID
        if key is not None:
            ids = np.asarray(self[key])
            cuts = np.flatnonzero(ids[1:] != ids[:-1]) + 1
        else:
            done = np.zeros(self.count, dtype=bool)
            for k in (self.TERMINATEDS, self.TRUNCATEDS):
                if k in self:
                    done |= np.asarray(self[k], dtype=bool)
            cuts = np.flatnonzero(done[:-1]) + 1
        bounds = [0, *cuts.tolist(), self.count]
        return [self.slice(a, b) for a, b in zip(bounds[:-1], bounds[1:]) if b > a]

    def timeslices(self, size: int) -> List["SampleBatch"]:
        return [self.slice(i, min(i + size, self.count)) for i in range(0, self.count, size)]

    def right_zero_pad(self, max_seq_len: int) -> "SampleBatch":
        pad = max_seq_len - self.count
        if pad <= 0:
            return self
        for k in list(self):
            v = np.asarray(self[k])
            if v.dtype == object:
                self[k] = np.concatenate([v, np.array([None] * pad, dtype=object)])
            else:
                self[k] = np.concatenate([v, np.zeros((pad,) + v.shape[1:], dtype=v.dtype)])
        self.count = max_seq_len
        return self

    def to_device(self, device, framework: str = "torch") -> "SampleBatch":
        import torch

        for k, v in list(self.items()):
            if isinstance(v, np.ndarray) and v.dtype != object:
                self[k] = torch.from_numpy(np.ascontiguousarray(v)).to(device, non_blocking=True)
        return self

    def size_bytes(self) -> int:
        return int(sum(getattr(v, "nbytes", 0) for v in self.values()))

    def as_multi_agent(self, module_id: str = "default_policy") -> "MultiAgentBatch":
        return MultiAgentBatch({module_id: self}, self.count)

    def __repr__(self):
        return f"SampleBatch({self.count}: {list(self.keys())})"


def concat_samples(samples: List) -> "SampleBatch | MultiAgentBatch":
    samples = [s for s in samples if s is not None and len(s) > 0] or samples[:1]
    if samples and isinstance(samples[0], MultiAgentBatch):
        return concat_samples_into_ma_batch(samples)
    if not samples:
        return SampleBatch()
    keys = list(samples[0].keys())
    return SampleBatch({k: np.concatenate([np.asarray(s[k]) for s in samples])
                        for k in keys if k != SampleBatch.SEQ_LENS})


class MultiAgentBatch:
    """Per-module SampleBatches of one sampling round (``policy_batches``) plus the env
    step count."""

    def __init__(self, policy_batches: Dict[str, SampleBatch], env_steps: int):
        self.policy_batches = dict(policy_batches)
        self.count = env_steps

    def env_steps(self) -> int:
        return self.count

    def agent_steps(self) -> int:
        return sum(len(b) for b in self.policy_batches.values())

    def __len__(self):
        return self.count

    @staticmethod
    def wrap_as_needed(policy_batches: Dict[str, SampleBatch], env_steps: int):
        if len(policy_batches) == 1 and "default_policy" in policy_batches:
            return policy_batches["default_policy"]
        return MultiAgentBatch(policy_batches, env_steps)

    def copy(self) -> "MultiAgentBatch":
        return MultiAgentBatch({k: v.copy() for k, v in self.policy_batches.items()}, self.count)

    def size_bytes(self) -> int:
        return sum(b.size_bytes() for b in self.policy_batches.values())

    def __repr__(self):
        return f"MultiAgentBatch({self.count} env steps: {list(self.policy_batches)})"


def concat_samples_into_ma_batch(samples: List) -> MultiAgentBatch:
    groups: Dict[str, List[SampleBatch]] = {}
    steps = 0
    for s in samples:
        if isinstance(s, SampleBatch):
            s = s.as_multi_agent()
        for k, b in s.policy_batches.items():
            groups.setdefault(k, []).append(b)
        steps += s.count
    return MultiAgentBatch({k: concat_samples(v) for k, v in groups.items()}, steps)


DEFAULT_POLICY_ID = "default_policy"
