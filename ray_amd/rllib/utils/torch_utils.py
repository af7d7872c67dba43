"""``ray.rllib.utils.torch_utils`` (reference path): torch helpers used by losses and
learners."""

from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as F

FLOAT_MIN = -3.4e38
FLOAT_MAX = 3.4e38


def apply_grad_clipping(optimizer, loss=None, grad_clip=None, grad_clip_by="global_norm"):
    """Clip the gradients of ``optimizer``'s parameters; returns {"grad_gnorm": ...}."""
    params = [p for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
    if not params or not grad_clip:
        return {}
    if grad_clip_by == "value":
        for p in params:
            p.grad.clamp_(-grad_clip, grad_clip)
        return {}
    n = torch.nn.utils.clip_grad_norm_(params, grad_clip)
    return {"grad_gnorm": float(n)}


def clip_gradients(gradients_dict: dict, *, grad_clip=None, grad_clip_by="value"):
    if grad_clip is None:
        return None
    grads = [g for g in gradients_dict.values() if g is not None]
    if grad_clip_by == "value":
        for g in grads:
            g.clamp_(-grad_clip, grad_clip)
        return None
    if grad_clip_by == "norm":
        for k, g in gradients_dict.items():
            if g is not None:
                n = g.norm()
                if n > grad_clip:
                    g.mul_(grad_clip / (n + 1e-6))
        return None
    total = global_norm(grads)
    if total > grad_clip:
        for g in grads:
            g.mul_(grad_clip / (total + 1e-6))
    return total


def global_norm(tensors: List[torch.Tensor]) -> torch.Tensor:
    return torch.sqrt(sum(torch.sum(t.float() ** 2) for t in tensors if t is not None))


def explained_variance(y, pred):
    var = torch.var(y)
    return torch.clamp(1 - torch.var(y - pred) / torch.clamp(var, min=1e-8), min=-1.0)


def huber_loss(x, delta: float = 1.0):
    return torch.where(x.abs() < delta, 0.5 * x ** 2, delta * (x.abs() - 0.5 * delta))


def l2_loss(x):
    return 0.5 * torch.sum(x ** 2)


def sequence_mask(lengths, maxlen: Optional[int] = None, dtype=None, time_major=False):
    lengths = torch.as_tensor(lengths)
    maxlen = int(maxlen or lengths.max())
    mask = torch.arange(maxlen, device=lengths.device)[None, :] < lengths[:, None]
    if time_major:
        mask = mask.t()
    return mask.to(dtype) if dtype is not None else mask


def reduce_mean_ignore_inf(x, axis: Optional[int] = None):
    mask = torch.ne(x, float("-inf"))
    xz = torch.where(mask, x, torch.zeros_like(x))
    return torch.sum(xz, axis) / torch.sum(mask.float(), axis)


def one_hot(x, space):
    n = getattr(space, "n", None)
    if n is not None:
        return F.one_hot(x.long(), n).float()
    nvec = getattr(space, "nvec", None)
    if nvec is not None:
        return torch.cat([F.one_hot(x[..., i].long(), int(k)).float()
                          for i, k in enumerate(nvec)], -1)
    raise ValueError(f"one_hot of unsupported space {space}")


def convert_to_torch_tensor(x, device=None, pin_memory: bool = False):
    if isinstance(x, dict):
        return {k: convert_to_torch_tensor(v, device, pin_memory) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(convert_to_torch_tensor(v, device, pin_memory) for v in x)
    if isinstance(x, torch.Tensor):
        t = x
    else:
        a = np.asarray(x)
        if a.dtype == object:
            return x
        t = torch.from_numpy(np.ascontiguousarray(a))
        if t.dtype == torch.float64:
            t = t.float()
    if pin_memory and t.device.type == "cpu" and torch.cuda.is_available():
        t = t.pin_memory()
    return t.to(device) if device is not None else t


def convert_to_non_torch_type(stats):
    from ray_amd.rllib.utils.numpy import convert_to_numpy

    return convert_to_numpy(stats, reduce_type=False)


def copy_torch_tensors(x, device=None):
    if isinstance(x, dict):
        return {k: copy_torch_tensors(v, device) for k, v in x.items()}
    if isinstance(x, torch.Tensor):
        return x.detach().clone().to(device) if device is not None else x.detach().clone()
    return x


def get_device(config, num_gpus_requested: int = 1):
    n = (config or {}).get("num_gpus_per_learner", 0) if isinstance(config, dict) else 0
    return torch.device("cuda", 0) if n and torch.cuda.is_available() else torch.device("cpu")


def set_torch_seed(seed: Optional[int] = None) -> None:
    if seed is not None:
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)


def softmax_cross_entropy_with_logits(logits, labels):
    return torch.sum(-labels * F.log_softmax(logits, -1), -1)


def atanh(x):
    return 0.5 * torch.log((1 + x).clamp(min=1e-7) / (1 - x).clamp(min=1e-7))
