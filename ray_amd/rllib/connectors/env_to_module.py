"""Env-to-module connectors (reference: rllib/connectors/env_to_module/
mean_std_filter.py, flatten_observations.py, prev_actions_prev_rewards.py;
rllib/utils/filter.py:181 MeanStdFilter).

MeanStdFilter on MI355X: the running mean/variance is owned by the LEARNER, which
updates it over each whole training batch with the HIP Welford kernel
(``ray_amd.ops.functional.RunningMeanStd``: obsnorm_update / obsnorm_apply) and
broadcasts it with the weights; EnvRunners only normalize with the latest stats and
record RAW observations, so the statistics see every sample exactly once and need no
per-runner delta merging.
"""

from __future__ import annotations

import numpy as np
import torch

from ray_amd.rllib.connectors.connector_v2 import ConnectorV2


class MeanStdFilter(ConnectorV2):
    """Normalize observations to zero mean / unit variance (clipped to +-clip)."""

    learner_side = True  # statistics are updated by the learner (HIP kernel on GPU)

    def __init__(self, input_observation_space=None, input_action_space=None, *,
                 clip: float = 10.0, eps: float = 1e-8, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.clip, self.eps = clip, eps
        self.rms = None

    def _ensure(self, shape):
        if self.rms is None:
            from ray_amd.ops.functional import RunningMeanStd

            self.rms = RunningMeanStd(shape, "cpu", clip=self.clip, eps=self.eps)

    def __call__(self, *, rl_module=None, batch, episodes=None, explore=True,
                 shared_data=None, **kw):
        obs = batch["obs"]
        self._ensure(obs.shape[1:])
        if self.rms.count > 1:
            x = torch.from_numpy(np.ascontiguousarray(obs, dtype=np.float32))
            batch["obs"] = self.rms.normalize(x).numpy()
        else:
            batch["obs"] = obs.astype(np.float32, copy=False)
        return batch

    def get_state(self):
        return self.rms.state_dict() if self.rms is not None else {}

    def set_state(self, state):
        if not state:
            return
        shape = tuple(state["mean"].shape)
        self._ensure(shape)
        self.rms.load_state_dict(state)


class FlattenObservations(ConnectorV2):
    def __call__(self, *, rl_module=None, batch, **kw):
        o = batch["obs"]
        batch["obs"] = o.reshape(o.shape[0], -1)
        return batch

    def recompute_output_observation_space(self, obs_space, act_space):
        from ray_amd.rllib.env.spaces import Box

        n = int(np.prod(obs_space.shape))
        return Box(-np.inf, np.inf, (n,), np.float32)


class PrevActionsPrevRewards(ConnectorV2):
    """Append the previous action (one-hot for discrete) and reward to the observation."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        o = batch["obs"].reshape(batch["obs"].shape[0], -1).astype(np.float32)
        pa = np.stack([e.prev_action for e in episodes]).astype(np.float32)
        pr = np.array([e.prev_reward for e in episodes], np.float32)[:, None]
        if pa.ndim == 1 and self.input_action_space is not None and \
                hasattr(self.input_action_space, "n"):
            oh = np.zeros((len(pa), self.input_action_space.n), np.float32)
            oh[np.arange(len(pa)), pa.astype(np.int64)] = 1.0
            pa = oh
        batch["obs"] = np.concatenate([o, pa.reshape(len(o), -1), pr], axis=1)
        return batch

    def recompute_output_observation_space(self, obs_space, act_space):
        from ray_amd.rllib.env.spaces import Box

        na = act_space.n if hasattr(act_space, "n") else int(np.prod(act_space.shape))
        n = int(np.prod(obs_space.shape)) + na + 1
        return Box(-np.inf, np.inf, (n,), np.float32)


def __getattr__(name):  # the pipeline pieces live in env_to_module_extra.py (imported lazily: no cycle)
    from ray_amd.rllib.connectors import env_to_module_extra as _x

    try:
        return getattr(_x, name)
    except AttributeError:
        raise AttributeError(name) from None
