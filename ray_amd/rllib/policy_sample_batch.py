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
        v = super().__getitem__(key)
        f = self.__dict__.get("_get_interceptor")
        return f(v) if f is not None else v

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

    # ------------------------------------------------------- reference helpers
    _training = False
    _slice_by_batch_id = False

    def is_training(self) -> bool:
        return bool(getattr(self, "_training", False))

    def set_training(self, training: bool = True) -> None:
        self._training = bool(training)

    def enable_slicing_by_batch_id(self) -> None:
        self._slice_by_batch_id = True

    def disable_slicing_by_batch_id(self) -> None:
        self._slice_by_batch_id = False

    def is_terminated_or_truncated(self) -> bool:
        """True when the last row ends an episode."""
        n = self.count
        if n == 0:
            return False
        t = self.get(self.TERMINATEDS)
        u = self.get(self.TRUNCATEDS)
        return bool((t is not None and t[-1]) or (u is not None and u[-1]))

    def is_single_trajectory(self) -> bool:
        """One episode, with no episode end before the last row."""
        eps = self.get(self.EPS_ID)
        if eps is not None and len(np.unique(eps)) > 1:
            return False
        for col in (self.TERMINATEDS, self.TRUNCATEDS):
            v = self.get(col)
            if v is not None and len(v) > 1 and np.any(np.asarray(v)[:-1]):
                return False
        return True

    def concat_samples(self, samples) -> "SampleBatch":
        return concat_samples(samples)

    def zero_pad(self, max_seq_len: int, exclude_states: bool = True) -> "SampleBatch":
        """In place: each sequence of ``seq_lens`` padded to ``max_seq_len`` rows."""
        lens = self.get(self.SEQ_LENS)
        if lens is None:
            return self.right_zero_pad(max_seq_len)
        lens = np.asarray(lens)
        for k, v in list(self.items()):
            if k == self.SEQ_LENS or (exclude_states and k.startswith("state_in")):
                continue
            v = np.asarray(v)
            out = np.zeros((len(lens) * max_seq_len,) + v.shape[1:], v.dtype)
            off = 0
            for i, ln in enumerate(lens):
                out[i * max_seq_len: i * max_seq_len + ln] = v[off:off + ln]
                off += ln
            dict.__setitem__(self, k, out)
        self.count = len(lens) * max_seq_len
        return self

    def compress(self, bulk: bool = False, columns=("obs", "new_obs")) -> "SampleBatch":
        """Observation columns as LZ4/zlib-compressed bytes (in place)."""
        import zlib

        for c in columns:
            if c in self and isinstance(self[c], np.ndarray):
                a = np.ascontiguousarray(self[c])
                blob = (a.dtype.str, a.shape, zlib.compress(a.tobytes(), 1))
                dict.__setitem__(self, c, _Compressed(blob))
        return self

    def decompress_if_needed(self, columns=("obs", "new_obs")) -> "SampleBatch":
        import zlib

        for c in columns:
            v = dict.get(self, c)
            if isinstance(v, _Compressed):
                dt, shape, data = v.blob
                dict.__setitem__(self, c, np.frombuffer(zlib.decompress(data),
                                                        dtype=np.dtype(dt)).reshape(shape))
        return self

    def set_get_interceptor(self, fn) -> None:
        """``fn(value)`` applied to every column read (e.g. a device transfer)."""
        self._get_interceptor = fn

    def get_single_step_input_dict(self, view_requirements=None, index="last") -> dict:
        """One row (the last, or ``index``) as a batch of size 1, ``new_obs`` as ``obs``."""
        i = self.count - 1 if index == "last" else int(index)
        out = {}
        for k, v in self.items():
            if k == self.SEQ_LENS:
                continue
            out[k] = np.asarray(v)[i:i + 1]
        if self.NEXT_OBS in out:
            out[self.OBS] = out[self.NEXT_OBS]
        return SampleBatch(out)

    def __repr__(self):
        return f"SampleBatch({self.count}: {list(self.keys())})"


class _Compressed:
    """A compressed column (dtype, shape, zlib bytes); ``len`` is its row count."""

    def __init__(self, blob):
        self.blob = blob

    def __len__(self):
        return int(self.blob[1][0]) if self.blob[1] else 0


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

    def timeslices(self, k: int) -> List["MultiAgentBatch"]:
        """Cut into batches of ``k`` env steps (each policy batch sliced alike)."""
        out = []
        for s in range(0, self.count, k):
            out.append(MultiAgentBatch({pid: b.slice(s, min(s + k, len(b)))
                                        for pid, b in self.policy_batches.items()
                                        if s < len(b)}, min(k, self.count - s)))
        return out

    @staticmethod
    def concat_samples(samples) -> "MultiAgentBatch":
        return concat_samples_into_ma_batch(samples)

    def compress(self, bulk: bool = False, columns=("obs", "new_obs")) -> "MultiAgentBatch":
        for b in self.policy_batches.values():
            b.compress(bulk, columns)
        return self

    def decompress_if_needed(self, columns=("obs", "new_obs")) -> "MultiAgentBatch":
        for b in self.policy_batches.values():
            b.decompress_if_needed(columns)
        return self

    def as_multi_agent(self) -> "MultiAgentBatch":
        return self

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
