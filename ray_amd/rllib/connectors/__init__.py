"""ConnectorV2 pipelines (reference: rllib/connectors/connector_v2.py,
connector_pipeline_v2.py, env_to_module/, module_to_env/, learner/)."""

from ray_amd.rllib.connectors.connector_v2 import ConnectorPipelineV2, ConnectorV2
from ray_amd.rllib.connectors.env_to_module import (FlattenObservations, MeanStdFilter,
                                                    PrevActionsPrevRewards)
from ray_amd.rllib.connectors.module_to_env import ClipActions, NormalizeAndClipActions

from ray_amd.rllib.connectors import common, learner  # noqa: F401,E402
from ray_amd.rllib.connectors.common import (AddObservationsFromEpisodesToBatch,  # noqa: E402,F401
                                             AddStatesFromEpisodesToBatch, AgentToModuleMapping,
                                             BatchIndividualItems, ModuleToAgentUnmapping,
                                             NumpyToTensor, TensorToNumpy)

__all__ = ["ConnectorV2", "ConnectorPipelineV2", "MeanStdFilter", "FlattenObservations",
           "PrevActionsPrevRewards", "ClipActions", "NormalizeAndClipActions"]
