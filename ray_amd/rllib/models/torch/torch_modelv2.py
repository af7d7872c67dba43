"""Old-stack custom models (reference: rllib/models/torch/torch_modelv2.py). A
``TorchModelV2`` maps ``input_dict["obs"]`` to ``num_outputs`` action-distribution inputs
and keeps a value head for ``value_function()``; registered with
``ModelCatalog.register_custom_model`` and named in ``model={"custom_model": ...}``, it
runs inside this framework's learners and env runners through an RLModule adapter."""

from __future__ import annotations

import torch.nn as nn


class TorchModelV2(nn.Module):
    def __init__(self, obs_space, action_space, num_outputs, model_config, name):
        nn.Module.__init__(self)
        self.obs_space = obs_space
        self.action_space = action_space
        self.num_outputs = num_outputs
        self.model_config = model_config
        self.name = name

    def forward(self, input_dict, state, seq_lens):
        """Returns ``(outputs [B, num_outputs], state)``."""
        raise NotImplementedError

    def value_function(self):
        """The value estimates [B] of the last ``forward`` call."""
        raise NotImplementedError

    def get_initial_state(self):
        return []

    def custom_loss(self, policy_loss, loss_inputs):
        return policy_loss

    def metrics(self):
        return {}
