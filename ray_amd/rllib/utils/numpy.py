"""``ray.rllib.utils.numpy`` (reference path): numpy helpers and constants."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.utils import (LARGE_INTEGER, MAX_LOG_NN_OUTPUT,  # noqa: F401
                                 MIN_LOG_NN_OUTPUT, SMALL_NUMBER, fc, lstm, one_hot, relu,
                                 sigmoid, softmax)

SMALL_NUMBER = SMALL_NUMBER


def convert_to_numpy(x, reduce_type: bool = True):
    """Nested structure of tensors -> numpy (float64 -> float32 with ``reduce_type``)."""
    if isinstance(x, dict):
        return {k: convert_to_numpy(v, reduce_type) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(convert_to_numpy(v, reduce_type) for v in x)
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    if reduce_type and isinstance(x, np.ndarray) and x.dtype == np.float64:
        x = x.astype(np.float32)
    return x


def flatten_inputs_to_1d_tensor(inputs, spaces_struct=None, time_axis: bool = False):
    """Concatenate the flattened leaves of a nested input along the last axis."""
    leaves = []

    def walk(v):
        if isinstance(v, dict):
            for k in sorted(v):
                walk(v[k])
        elif isinstance(v, (list, tuple)):
            for x in v:
                walk(x)
        else:
            a = np.asarray(v, dtype=np.float32)
            lead = 2 if time_axis else 1
            leaves.append(a.reshape(a.shape[:lead] + (-1,)))
    walk(inputs)
    return np.concatenate(leaves, axis=-1)


def make_action_immutable(obj):
    if isinstance(obj, np.ndarray):
        obj.setflags(write=False)
    elif isinstance(obj, dict):
        for v in obj.values():
            make_action_immutable(v)
    return obj


def huber_loss(x, delta: float = 1.0):
    x = np.asarray(x, np.float64)
    return np.where(np.abs(x) < delta, 0.5 * x ** 2, delta * (np.abs(x) - 0.5 * delta))


def l2_loss(x):
    return np.sum(np.square(x)) / 2.0
