"""``ModelV2`` (reference: python/ray/rllib/models/modelv2.py): the framework-neutral base of
old-stack custom models. ray_amd is torch-only, so the base is ``TorchModelV2`` and
``ModelV2`` names the interface (``forward(input_dict, state, seq_lens)``,
``value_function()``, ``get_initial_state()``)."""

from ray_amd.rllib.models.torch.torch_modelv2 import TorchModelV2

ModelV2 = TorchModelV2


def restore_original_dimensions(obs, obs_space, tensorlib="torch"):
    """Observations arrive unflattened in ray_amd (the encoders flatten): identity."""
    return obs
