"""Env-to-module pipeline pieces beyond the filters (reference:
python/ray/rllib/connectors/env_to_module/__init__.py)."""

from __future__ import annotations

from ray_amd.rllib.connectors.common import (AddObservationsFromEpisodesToBatch,  # noqa: F401
                                             AddStatesFromEpisodesToBatch, AgentToModuleMapping,
                                             BatchIndividualItems, NumpyToTensor)
from ray_amd.rllib.connectors.connector_v2 import ConnectorPipelineV2, ConnectorV2
from ray_amd.rllib.connectors.env_to_module import PrevActionsPrevRewards


class EnvToModulePipeline(ConnectorPipelineV2):
    """The env -> module pipeline of an EnvRunner."""


PrevActionsPrevRewardsConnector = PrevActionsPrevRewards


class WriteObservationsToEpisodes(ConnectorV2):
    """The runner records each step's (raw) observation in its episodes itself."""

    def __call__(self, *, rl_module=None, batch, **kw):
        return batch
