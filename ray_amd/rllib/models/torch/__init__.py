from ray_amd.rllib.models.torch.torch_modelv2 import TorchModelV2  # noqa: F401
