"""Debug helpers (reference: rllib/utils/debug/): ``summarize`` pretty-prints nested
structures of arrays by shape/dtype/stats instead of their contents."""

from __future__ import annotations

import pprint

import numpy as np


def _summ(x):
    if isinstance(x, dict):
        return {k: _summ(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_summ(v) for v in x)
    if hasattr(x, "detach") and hasattr(x, "cpu"):
        x = x.detach().cpu().numpy()
    if isinstance(x, np.ndarray):
        if x.size == 0:
            return f"np.ndarray({x.shape}, dtype={x.dtype})"
        if np.issubdtype(x.dtype, np.number):
            return (f"np.ndarray({x.shape}, dtype={x.dtype}, min={x.min():.3g}, "
                    f"max={x.max():.3g}, mean={x.mean():.3g})")
        return f"np.ndarray({x.shape}, dtype={x.dtype}, head={list(x.reshape(-1)[:3])})"
    return x


def summarize(obj) -> str:
    return pprint.pformat(_summ(obj))


def update_global_seed_if_necessary(framework=None, seed=None) -> None:
    if seed is None:
        return
    import random

    import torch

    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
