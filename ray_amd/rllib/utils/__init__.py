"""``ray.rllib.utils`` (reference: python/ray/rllib/utils/__init__.py): small helpers that
user code imports from RLlib — dict utilities, numpy NN ops, the ``check`` comparison used
by tests, framework imports, schedules and observation filters."""

from __future__ import annotations

import functools
import warnings
from typing import Any, List, Optional

import numpy as np

from ray_amd.rllib.utils.filter import Filter, MeanStdFilter, NoFilter  # noqa: F401
from ray_amd.rllib.utils.filter_manager import FilterManager  # noqa: F401
from ray_amd.rllib.utils.schedules import (ConstantSchedule, ExponentialSchedule,  # noqa: F401
                                           LinearSchedule, PiecewiseSchedule,
                                           PolynomialSchedule)
from ray_amd.tune.utils import deep_update, merge_dicts  # noqa: F401
from ray_amd.util.annotations import DeveloperAPI, PublicAPI  # noqa: F401

LARGE_INTEGER = 100000000
MIN_LOG_NN_OUTPUT = -5
MAX_LOG_NN_OUTPUT = 2
SMALL_NUMBER = 1e-6


def override(parent_cls):
    """Marks a method as overriding one of ``parent_cls`` (checked at definition)."""

    def check(method):
        if not hasattr(parent_cls, method.__name__):
            raise NameError(f"{method.__name__} does not override any method of "
                            f"{parent_cls.__name__}")
        return method

    return check


def force_list(elements=None, to_tuple: bool = False):
    ctor = tuple if to_tuple else list
    if elements is None:
        return ctor()
    if isinstance(elements, (list, tuple, set, frozenset)) or (
            hasattr(elements, "__iter__") and not isinstance(elements, (str, bytes, dict))
            and not hasattr(elements, "shape")):
        return ctor(elements)
    return ctor([elements])


force_tuple = functools.partial(force_list, to_tuple=True)


def add_mixins(base, mixins, reversed: bool = False):
    """A subclass of ``base`` with ``mixins`` mixed in (first mixin highest priority)."""
    mixins = list(mixins or [])
    if reversed:
        mixins = mixins[::-1]
    bases = tuple(mixins) + (base,)
    return type(base.__name__, bases, {})


def deprecation_warning(old: str, new: Optional[str] = None, *, help: Optional[str] = None,
                        error: bool = False) -> None:
    msg = f"`{old}` has been deprecated." + (f" Use `{new}` instead." if new else "") + \
        (f" {help}" if help else "")
    if error:
        raise ValueError(msg)
    warnings.warn(msg, DeprecationWarning, stacklevel=2)


def try_import_torch(error: bool = False):
    try:
        import torch
        import torch.nn as nn
        return torch, nn
    except ImportError:
        if error:
            raise
        return None, None


def try_import_tf(error: bool = False):
    """(tf1, tf, version): TensorFlow is not part of this framework's stack."""
    if error:
        raise ImportError("TensorFlow is not installed")
    return None, None, None


def try_import_tfp(error: bool = False):
    if error:
        raise ImportError("tensorflow_probability is not installed")
    return None


def try_import_jax(error: bool = False):
    try:
        import flax  # noqa: F401
        import jax
        return jax, flax
    except ImportError:
        if error:
            raise
        return None, None


def framework_iterator(config=None, frameworks=("torch",), session: bool = False, **kw):
    """Yields each framework to test under; ray_amd is torch-only."""
    for fw in frameworks if isinstance(frameworks, (list, tuple)) else [frameworks]:
        if fw != "torch":
            continue
        if config is not None:
            if hasattr(config, "framework"):
                config.framework("torch")
            elif isinstance(config, dict):
                config["framework"] = "torch"
        yield fw


# ----------------------------------------------------------------- numpy NN ops
def sigmoid(x, derivative: bool = False):
    s = 1.0 / (1.0 + np.exp(-np.asarray(x, dtype=np.float64)))
    return s * (1 - s) if derivative else s


def relu(x, alpha: float = 0.0):
    x = np.asarray(x)
    return np.maximum(x, x * alpha)


def softmax(x, axis: int = -1, epsilon: Optional[float] = None):
    x = np.asarray(x, dtype=np.float64)
    e = np.exp(x - np.max(x, axis=axis, keepdims=True))
    out = e / np.sum(e, axis=axis, keepdims=True)
    return np.maximum(out, epsilon if epsilon is not None else SMALL_NUMBER)


def one_hot(x, depth: int = 0, on_value: float = 1.0, off_value: float = 0.0,
            dtype=np.float32):
    x = np.asarray(x)
    depth = depth or int(np.max(x)) + 1
    out = np.full(x.shape + (depth,), off_value, dtype=dtype)
    np.put_along_axis(out, x[..., None].astype(np.int64), on_value, axis=-1)
    return out


def fc(x, weights, biases=None, framework=None):
    """Dense layer ``x @ weights + biases`` (weights [in, out])."""
    out = np.matmul(np.asarray(x), np.asarray(weights))
    return out + np.asarray(biases) if biases is not None else out


def lstm(x, weights, biases=None, initial_internal_states=None, time_major: bool = False,
         forget_bias: float = 1.0):
    """A numpy LSTM over [B, T, in] (``weights`` [in + units, 4 units], gate order
    i, j(c~), f, o as in the reference); returns (outputs, (c, h))."""
    x = np.asarray(x, dtype=np.float64)
    if time_major:
        x = np.transpose(x, (1, 0, 2))
    B, T, _ = x.shape
    units = weights.shape[1] // 4
    c = np.zeros((B, units)) if initial_internal_states is None else \
        np.asarray(initial_internal_states[0], dtype=np.float64)
    h = np.zeros((B, units)) if initial_internal_states is None else \
        np.asarray(initial_internal_states[1], dtype=np.float64)
    outs = np.zeros((B, T, units))
    for t in range(T):
        z = np.concatenate([x[:, t], h], axis=1) @ weights
        if biases is not None:
            z = z + biases
        i, j, f, o = np.split(z, 4, axis=1)
        c = sigmoid(f + forget_bias) * c + sigmoid(i) * np.tanh(j)
        h = sigmoid(o) * np.tanh(c)
        outs[:, t] = h
    if time_major:
        outs = np.transpose(outs, (1, 0, 2))
    return outs, (c, h)


# ----------------------------------------------------------------- test helpers
def check(x, y, decimals: int = 5, atol: Optional[float] = None,
          rtol: Optional[float] = None, false: bool = False):
    """Assert that nested structures ``x`` and ``y`` are equal (floats to ``decimals``
    places, or ``atol``/``rtol``); ``false=True`` asserts they differ."""
    def _eq(a, b):
        if isinstance(a, dict):
            if not isinstance(b, dict) or set(a) != set(b):
                return False
            return all(_eq(a[k], b[k]) for k in a)
        if isinstance(a, (list, tuple)) and not isinstance(b, np.ndarray):
            return isinstance(b, (list, tuple)) and len(a) == len(b) and \
                all(_eq(p, q) for p, q in zip(a, b))
        if hasattr(a, "detach"):
            a = a.detach().cpu().numpy()
        if hasattr(b, "detach"):
            b = b.detach().cpu().numpy()
        a, b = np.asarray(a), np.asarray(b)
        if a.shape != b.shape:
            return False
        if a.dtype.kind in "fc" or b.dtype.kind in "fc":
            if atol is not None or rtol is not None:
                return bool(np.allclose(a, b, atol=atol or 0.0, rtol=rtol or 0.0,
                                        equal_nan=True))
            return bool(np.allclose(a, b, atol=0.5 * 10 ** -decimals, rtol=0,
                                    equal_nan=True))
        return bool(np.array_equal(a, b))

    same = _eq(x, y)
    if false and same:
        raise AssertionError(f"{x!r} and {y!r} are equal (expected them to differ)")
    if not false and not same:
        raise AssertionError(f"{x!r} != {y!r}")


def check_train_results(train_results: dict) -> dict:
    """Assert the standard keys of an ``Algorithm.train()`` result."""
    for key in ("training_iteration", "time_total_s", "env_runners", "learners",
                "num_env_steps_sampled_lifetime"):
        if key not in train_results:
            raise AssertionError(f"'{key}' not found in train results")
    if not isinstance(train_results["training_iteration"], int):
        raise AssertionError("training_iteration must be an int")
    return train_results


def check_compute_single_action(algorithm, include_state: bool = False,
                                include_prev_action_reward: bool = False) -> None:
    """``compute_single_action`` returns an action in the action space, explore on/off."""
    obs = algorithm.observation_space.sample()
    for explore in (True, False):
        a = algorithm.compute_single_action(obs, explore=explore)
        if isinstance(a, tuple):
            a = a[0]
        if not algorithm.action_space.contains(a):
            raise AssertionError(f"action {a!r} not in {algorithm.action_space}")


__all__ = ["add_mixins", "check", "check_compute_single_action", "check_train_results",
           "deep_update", "deprecation_warning", "fc", "force_list", "force_tuple",
           "framework_iterator", "lstm", "merge_dicts", "one_hot", "override", "relu",
           "sigmoid", "softmax", "try_import_jax", "try_import_tf", "try_import_tfp",
           "try_import_torch", "ConstantSchedule", "DeveloperAPI", "ExponentialSchedule",
           "Filter", "FilterManager", "LARGE_INTEGER", "LinearSchedule", "MAX_LOG_NN_OUTPUT",
           "MIN_LOG_NN_OUTPUT", "PiecewiseSchedule", "PolynomialSchedule", "PublicAPI",
           "SMALL_NUMBER"]
