"""``ray.rllib.utils.framework`` (reference path): framework imports. ray_amd's RLlib is
torch-only; the TF / JAX probes return None."""

from ray_amd.rllib.utils import (try_import_jax, try_import_tf,  # noqa: F401
                                 try_import_tfp, try_import_torch)


def get_variable(value, framework: str = "torch", trainable: bool = False, tf_name=None,
                 torch_tensor: bool = False, device=None, shape=None, dtype=None):
    import numpy as np
    import torch

    if torch_tensor or framework == "torch":
        t = torch.as_tensor(np.asarray(value) if shape is None else np.full(shape, value),
                            dtype=dtype if isinstance(dtype, torch.dtype) else None)
        if trainable:
            t = torch.nn.Parameter(t.float())
        return t.to(device) if device is not None else t
    return value


def get_activation_fn(name=None, framework: str = "torch"):
    import torch.nn as nn

    if name in (None, "linear"):
        return None
    table = {"relu": nn.ReLU, "tanh": nn.Tanh, "elu": nn.ELU, "swish": nn.SiLU,
             "silu": nn.SiLU, "sigmoid": nn.Sigmoid, "gelu": nn.GELU, "leaky_relu": nn.LeakyReLU}
    if name not in table:
        raise ValueError(f"Unknown activation ({name}) for framework={framework}")
    return table[name]
