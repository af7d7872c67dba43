"""Connector pieces used on both sides (reference: python/ray/rllib/connectors/common/):
batching, tensor conversion, agent <-> module mapping.

ray_amd's EnvRunners step their envs in lock-step, so a connector batch is already a dict
of arrays with the env index leading (``connector_v2.py``). These pieces make the
reference's pipelines compose: they add what is missing and leave present columns alone."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.connectors.connector_v2 import ConnectorV2


class AddObservationsFromEpisodesToBatch(ConnectorV2):
    """``batch["obs"]`` from each episode's latest observation, when not there yet."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        if "obs" not in batch and episodes:
            batch["obs"] = np.stack([np.asarray(_last_obs(e)) for e in episodes])
        return batch


def _last_obs(ep):
    if hasattr(ep, "get_observations"):
        return ep.get_observations(-1)
    if hasattr(ep, "observations"):
        return ep.observations[-1]
    return getattr(ep, "obs")


class AddStatesFromEpisodesToBatch(ConnectorV2):
    """Recurrent state inputs: the runner keeps each env's state and adds
    ``state_in_*`` itself; for a stateless module there is nothing to add."""

    def __call__(self, *, rl_module=None, batch, episodes=None, **kw):
        return batch


class BatchIndividualItems(ConnectorV2):
    """Lists of per-env items -> one stacked array per column."""

    def __call__(self, *, rl_module=None, batch, **kw):
        for k, v in list(batch.items()):
            if isinstance(v, list) and v and not isinstance(v[0], (str, bytes)):
                try:
                    batch[k] = np.stack([np.asarray(x) for x in v])
                except ValueError:
                    pass
        return batch


class NumpyToTensor(ConnectorV2):
    """numpy columns -> torch tensors (on the module's device, or ``device``)."""

    def __init__(self, input_observation_space=None, input_action_space=None, *,
                 as_learner_connector: bool = False, pin_memory: bool = False, device=None,
                 **kw):
        super().__init__(input_observation_space, input_action_space)
        self.pin_memory, self.device = pin_memory, device

    def __call__(self, *, rl_module=None, batch, **kw):
        import torch

        dev = self.device
        if dev is None and rl_module is not None:
            p = next(iter(rl_module.parameters()), None) if hasattr(rl_module,
                                                                    "parameters") else None
            dev = p.device if p is not None else None
        for k, v in list(batch.items()):
            if isinstance(v, np.ndarray) and v.dtype.kind in "biuf":
                t = torch.from_numpy(np.ascontiguousarray(v))
                if self.pin_memory and torch.cuda.is_available():
                    t = t.pin_memory()
                batch[k] = t.to(dev, non_blocking=True) if dev is not None else t
        return batch


class TensorToNumpy(ConnectorV2):
    def __call__(self, *, rl_module=None, batch, **kw):
        for k, v in list(batch.items()):
            if hasattr(v, "detach"):
                batch[k] = v.detach().cpu().numpy()
        return batch


class AgentToModuleMapping(ConnectorV2):
    """Single-agent lock-step batches map 1:1 to the default module; multi-agent runners
    (env/multi_agent_env_runner.py) group per module themselves."""

    def __init__(self, input_observation_space=None, input_action_space=None, *,
                 rl_module_specs=None, agent_to_module_mapping_fn=None, **kw):
        super().__init__(input_observation_space, input_action_space)
        self.agent_to_module_mapping_fn = agent_to_module_mapping_fn

    def __call__(self, *, rl_module=None, batch, **kw):
        return batch


class ModuleToAgentUnmapping(ConnectorV2):
    def __call__(self, *, rl_module=None, batch, **kw):
        return batch
