"""Module-to-env connectors (reference: rllib/connectors/module_to_env/
normalize_and_clip_actions.py)."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.connectors.connector_v2 import ConnectorV2


class ClipActions(ConnectorV2):
    """Clip continuous actions into the action space bounds before env.step."""

    def __call__(self, *, rl_module=None, batch, **kw):
        sp = self.input_action_space
        if sp is not None and hasattr(sp, "low"):
            batch["actions_for_env"] = np.clip(batch.get("actions_for_env", batch["actions"]),
                                               sp.low, sp.high)
        return batch


class NormalizeAndClipActions(ConnectorV2):
    """Map module outputs in [-1, 1] to the action space bounds (then clip)."""

    def __call__(self, *, rl_module=None, batch, **kw):
        sp = self.input_action_space
        if sp is not None and hasattr(sp, "low"):
            a = np.clip(batch.get("actions_for_env", batch["actions"]), -1.0, 1.0)
            batch["actions_for_env"] = sp.low + (a + 1.0) * 0.5 * (sp.high - sp.low)
        return batch


def __getattr__(name):  # the pipeline pieces live in module_to_env_extra.py (imported lazily: no cycle)
    from ray_amd.rllib.connectors import module_to_env_extra as _x

    try:
        return getattr(_x, name)
    except AttributeError:
        raise AttributeError(name) from None
