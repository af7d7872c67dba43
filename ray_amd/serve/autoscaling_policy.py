"""Serve autoscaling decisions as a pure function (reference:
python/ray/serve/autoscaling_policy.py ``replica_queue_length_autoscaling_policy``).

The controller (``_controller.ServeController._autoscale``) averages the load (requests
ongoing at replicas + queued at handles) over ``look_back_period_s`` and calls the
deployment's policy once per control-loop tick with the reference's keyword arguments::

    policy(curr_target_num_replicas=..., total_num_requests=..., num_running_replicas=...,
           config=..., capacity_adjusted_min_replicas=..., capacity_adjusted_max_replicas=...,
           policy_state=...)

``config`` is the controller's autoscaling dict (or an ``AutoscalingConfig``);
``policy_state`` is a dict kept per deployment between calls, holding ``now`` (the
controller's clock) plus whatever the policy stores. A custom policy is set with
``autoscaling_config={"policy": fn_or_import_path, ...}`` (``_policy`` is accepted too).

The default policy here counts the delays in seconds of the controller clock rather than
in control-loop periods, so a decision needs ``upscale_delay_s`` / ``downscale_delay_s``
of consistent signal regardless of the tick rate.
"""

from __future__ import annotations

import importlib
import math
import time
from typing import Any, Callable, Dict, Optional


def _get(config, key, default=None):
    if config is None:
        return default
    if isinstance(config, dict):
        v = config.get(key, default)
    else:
        v = getattr(config, key, default)
    return default if v is None else v


def _target(config) -> float:
    if config is not None and not isinstance(config, dict) and \
            hasattr(config, "get_target_ongoing_requests"):
        return config.get_target_ongoing_requests()
    return float(_get(config, "target_ongoing_requests",
                      _get(config, "target_num_ongoing_requests_per_replica", 2)))


def _calculate_desired_num_replicas(config, total_num_requests: float,
                                    num_running_replicas: int,
                                    override_min_replicas: Optional[float] = None,
                                    override_max_replicas: Optional[float] = None) -> int:
    """Replicas that would carry ``total_num_requests`` at the target per replica, moved
    only ``upscaling_factor`` / ``downscaling_factor`` of the way from the current count,
    clamped to [min, max]."""
    lo = override_min_replicas if override_min_replicas is not None else \
        _get(config, "min_replicas", 1)
    hi = override_max_replicas if override_max_replicas is not None else \
        _get(config, "max_replicas", 10)
    cur = num_running_replicas
    if total_num_requests > 1e-9:
        desired = math.ceil(total_num_requests / max(_target(config), 1e-9))
    else:
        desired = lo
    up = _get(config, "upscaling_factor")
    down = _get(config, "downscaling_factor")
    if desired > cur and up:
        desired = cur + math.ceil((desired - cur) * up)
    elif desired < cur and down:
        desired = cur - max(1, math.floor((cur - desired) * down))
    return int(max(lo, min(hi, desired)))


def replica_queue_length_autoscaling_policy(
        curr_target_num_replicas: int, total_num_requests: float,
        num_running_replicas: int, config, capacity_adjusted_min_replicas: int,
        capacity_adjusted_max_replicas: int, policy_state: Dict[str, Any]) -> int:
    """The default policy: scale toward ``total_num_requests / target_ongoing_requests``
    once the same direction has held for the configured delay."""
    now = policy_state.get("now", time.time())
    desired = _calculate_desired_num_replicas(
        config, total_num_requests, curr_target_num_replicas,
        capacity_adjusted_min_replicas, capacity_adjusted_max_replicas)
    decision = curr_target_num_replicas
    if desired > curr_target_num_replicas:
        policy_state["under_since"] = None
        since = policy_state.get("over_since") or now
        policy_state["over_since"] = since
        if now - since >= float(_get(config, "upscale_delay_s", 30.0)):
            decision = desired
            policy_state["over_since"] = None
    elif desired < curr_target_num_replicas:
        policy_state["over_since"] = None
        since = policy_state.get("under_since") or now
        policy_state["under_since"] = since
        if now - since >= float(_get(config, "downscale_delay_s", 600.0)):
            decision = desired
            policy_state["under_since"] = None
            policy_state["reset_samples"] = True
    else:
        policy_state["over_since"] = policy_state["under_since"] = None
    return decision


default_autoscaling_policy = replica_queue_length_autoscaling_policy
DEFAULT_AUTOSCALING_POLICY = "ray_amd.serve.autoscaling_policy:default_autoscaling_policy"


def resolve_policy(policy) -> Callable:
    """A policy callable from a callable, ``"pkg.mod:fn"`` / ``"pkg.mod.fn"``, or None."""
    if policy is None or policy == "":
        return default_autoscaling_policy
    if callable(policy):
        return policy
    path = str(policy)
    mod, _, attr = path.partition(":") if ":" in path else path.rpartition(".")
    fn = getattr(importlib.import_module(mod), attr)
    if not callable(fn):
        raise TypeError(f"autoscaling policy {path!r} is not callable")
    return fn
