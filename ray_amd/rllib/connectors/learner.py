"""Learner connector pieces (reference: python/ray/rllib/connectors/learner/): they turn
episodes / sampled columns into the train batch. ray_amd's learners build the batch from
the runners' column stores (GAE and returns run as HIP kernels inside the learner step);
these pieces serve reference-style custom learner pipelines."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.connectors.common import (AddObservationsFromEpisodesToBatch,  # noqa: F401
                                             AddStatesFromEpisodesToBatch, AgentToModuleMapping,
                                             BatchIndividualItems, NumpyToTensor)
from ray_amd.rllib.connectors.connector_v2 import ConnectorPipelineV2, ConnectorV2


class LearnerConnectorPipeline(ConnectorPipelineV2):
    """The episodes -> train-batch pipeline of a Learner."""


class AddColumnsFromEpisodesToTrainBatch(ConnectorV2):
    """rewards / actions / terminateds / truncateds / action_logp columns from episodes
    (``SingleAgentEpisode.get_sample_batch``), concatenated over episodes."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        if not episodes:
            return batch
        parts = [e.get_sample_batch() for e in episodes if hasattr(e, "get_sample_batch")]
        for col in ("actions", "rewards", "terminateds", "truncateds", "action_logp",
                    "action_dist_inputs"):
            if col not in batch and parts and all(col in p for p in parts):
                batch[col] = np.concatenate([np.asarray(p[col]) for p in parts])
        return batch


class AddNextObservationsFromEpisodesToTrainBatch(ConnectorV2):
    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        if "next_obs" in batch or not episodes:
            return batch
        parts = [e.get_sample_batch() for e in episodes if hasattr(e, "get_sample_batch")]
        if parts and all("next_obs" in p for p in parts):
            batch["next_obs"] = np.concatenate([np.asarray(p["next_obs"]) for p in parts])
        return batch


class AddOneTsToEpisodesAndTruncate(ConnectorV2):
    """The reference extends each episode by one artificial step for value bootstrapping;
    ray_amd's runners ship the bootstrap observation (``next_obs``) instead."""

    def __call__(self, *, rl_module=None, batch, **kw):
        return batch


class GeneralAdvantageEstimation(ConnectorV2):
    """GAE over time-major columns ``rewards``, ``vf_preds``, ``terminateds`` (and an
    optional ``bootstrap_value``): adds ``advantages`` and ``value_targets`` (numpy; the
    learner's own path runs the HIP GAE kernel)."""

    def __init__(self, input_observation_space=None, input_action_space=None, *,
                 gamma: float = 0.99, lambda_: float = 1.0, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.gamma, self.lambda_ = gamma, lambda_

    def __call__(self, *, rl_module=None, batch, **kw):
        r = np.asarray(batch["rewards"], np.float64)
        v = np.asarray(batch["vf_preds"], np.float64)
        d = np.asarray(batch["terminateds"], np.float64)
        boot = np.asarray(batch.get("bootstrap_value", np.zeros(r.shape[1:])), np.float64)
        adv = np.zeros_like(r)
        last = np.zeros(r.shape[1:])
        for t in range(len(r) - 1, -1, -1):
            nv = boot if t == len(r) - 1 else v[t + 1]
            delta = r[t] + self.gamma * nv * (1 - d[t]) - v[t]
            last = delta + self.gamma * self.lambda_ * (1 - d[t]) * last
            adv[t] = last
        batch["advantages"] = adv.astype(np.float32)
        batch["value_targets"] = (adv + v).astype(np.float32)
        return batch
