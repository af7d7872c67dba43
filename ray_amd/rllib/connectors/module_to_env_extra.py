"""Module-to-env pipeline pieces (reference: python/ray/rllib/connectors/module_to_env/)."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.connectors.common import ModuleToAgentUnmapping, TensorToNumpy  # noqa: F401
from ray_amd.rllib.connectors.connector_v2 import ConnectorPipelineV2, ConnectorV2


class ModuleToEnvPipeline(ConnectorPipelineV2):
    """The module -> env pipeline of an EnvRunner."""


class GetActions(ConnectorV2):
    """Sample ``actions`` (and ``action_logp``) from ``action_dist_inputs`` when the
    module returned only the distribution inputs."""

    def __call__(self, *, rl_module=None, batch, explore=True, **kw):
        if "actions" in batch or "action_dist_inputs" not in batch:
            return batch
        import torch

        di = batch["action_dist_inputs"]
        di = di if isinstance(di, torch.Tensor) else torch.as_tensor(np.asarray(di))
        if rl_module is not None and hasattr(rl_module, "sample_actions"):
            a, lp = rl_module.sample_actions(di.float(), explore)
        else:  # categorical logits
            dist = torch.distributions.Categorical(logits=di.float())
            a = dist.sample() if explore else di.argmax(-1)
            lp = dist.log_prob(a)
        batch["actions"], batch["action_logp"] = a, lp
        return batch


class UnBatchToIndividualItems(ConnectorV2):
    """Per-env rows of the batched actions (the env-facing form of ``actions_for_env``)."""

    def __call__(self, *, rl_module=None, batch, **kw):
        a = batch.get("actions_for_env", batch.get("actions"))
        if a is not None and not isinstance(a, list):
            batch["actions_for_env"] = list(np.asarray(a))
        return batch


class ListifyDataForVectorEnv(UnBatchToIndividualItems):
    pass


class RemoveSingleTsTimeRankFromBatch(ConnectorV2):
    """Drop a time axis of length 1 (recurrent modules' single-step outputs)."""

    def __call__(self, *, rl_module=None, batch, **kw):
        for k, v in list(batch.items()):
            shp = getattr(v, "shape", None)
            if shp is not None and len(shp) >= 2 and shp[1] == 1 and k != "obs":
                batch[k] = v[:, 0]
        return batch
