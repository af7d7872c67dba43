"""SampleBatch / MultiAgentBatch (reference: rllib/policy/tests/test_sample_batch.py)."""

import numpy as np
import pytest

from ray_amd.rllib import MultiAgentBatch, SampleBatch, concat_samples


def _sb(n, eps, start=0):
    return SampleBatch({SampleBatch.OBS: np.arange(start, start + n, dtype=np.float32),
                        SampleBatch.REWARDS: np.ones(n), SampleBatch.EPS_ID: np.array(eps),
                        SampleBatch.TERMINATEDS: np.array([i == n - 1 for i in range(n)])})


def test_concat_slice_shuffle_split():
    a, b = _sb(3, [0, 0, 1]), _sb(2, [1, 2], start=3)
    c = concat_samples([a, b])
    assert len(c) == 5 and c[SampleBatch.OBS].tolist() == [0, 1, 2, 3, 4]
    assert c[1:3][SampleBatch.OBS].tolist() == [1, 2]
    eps = c.split_by_episode()
    assert [len(e) for e in eps] == [2, 2, 1]
    assert [len(t) for t in c.timeslices(2)] == [2, 2, 1]
    rows = list(c.rows())
    assert rows[4][SampleBatch.EPS_ID] == 2
    s = c.copy().shuffle(seed=0)
    assert sorted(s[SampleBatch.OBS].tolist()) == [0, 1, 2, 3, 4]
    padded = _sb(2, [5, 5]).right_zero_pad(4)
    assert len(padded) == 4 and padded[SampleBatch.OBS].tolist() == [0, 1, 0, 0]
    with pytest.raises(ValueError):
        SampleBatch({"a": np.zeros(2), "b": np.zeros(3)})
    t = c.copy().to_device("cpu")
    assert t[SampleBatch.OBS].shape == (5,)


def test_multi_agent_batch():
    ma1 = MultiAgentBatch({"p0": _sb(2, [0, 0]), "p1": _sb(3, [1, 1, 1])}, env_steps=3)
    ma2 = _sb(1, [7]).as_multi_agent("p0")
    m = concat_samples([ma1, ma2])
    assert isinstance(m, MultiAgentBatch) and m.env_steps() == 4
    assert len(m.policy_batches["p0"]) == 3 and m.agent_steps() == 6
    assert isinstance(MultiAgentBatch.wrap_as_needed({"default_policy": _sb(1, [0])}, 1),
                      SampleBatch)
