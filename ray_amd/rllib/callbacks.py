"""RLlib callbacks and custom metrics.

API contract (reference: rllib/algorithms/callbacks.py:43 ``RLlibCallback`` /
``DefaultCallbacks`` — ``on_algorithm_init``, ``on_train_result``,
``on_evaluate_start``/``on_evaluate_end``, ``on_checkpoint_loaded``,
``on_environment_created``, ``on_episode_created``/``on_episode_start``/
``on_episode_step``/``on_episode_end``, ``on_sample_end``; plus a metrics logger).

Design: episode hooks run inside the EnvRunner actors (one ``EpisodeState`` per env
slot, passed to the hooks); values a callback logs with ``metrics_logger.log_value``
(or writes into ``episode.custom_metrics``) are reduced per runner, shipped with the
runner metrics and averaged into ``result["env_runners"]["custom_metrics"]``.
"""

from __future__ import annotations

import numpy as np


class MetricsLogger:
    """Minimal reduce-on-read metric store (reference: rllib/utils/metrics/
    metrics_logger.py)."""

    def __init__(self):
        self.values: dict = {}
        self.reduce: dict = {}

    def log_value(self, key, value, reduce: str = "mean", **kw):
        self.values.setdefault(key, []).append(float(value))
        self.reduce[key] = reduce

    def peek(self, key, default=None):
        vs = self.values.get(key)
        if not vs:
            return default
        return _reduce(vs, self.reduce.get(key, "mean"))

    def reduce_all(self, clear: bool = True) -> dict:
        out = {k: _reduce(v, self.reduce.get(k, "mean")) for k, v in self.values.items() if v}
        if clear:
            self.values = {}
        return out


def _reduce(vs, how):
    if how == "sum":
        return float(np.sum(vs))
    if how == "max":
        return float(np.max(vs))
    if how == "min":
        return float(np.min(vs))
    return float(np.mean(vs))


class EpisodeState:
    """The episode of one env slot as seen by callbacks and connectors."""

    __slots__ = ("id_", "env_index", "t", "total_reward", "prev_action", "prev_reward",
                 "custom_metrics", "user_data", "worker_index")

    def __init__(self, env_index, worker_index, act_dummy):
        self.env_index = env_index
        self.worker_index = worker_index
        self.reset(act_dummy, 0)

    def reset(self, act_dummy, eid):
        self.id_ = eid
        self.t = 0
        self.total_reward = 0.0
        self.prev_action = act_dummy
        self.prev_reward = 0.0
        self.custom_metrics = {}
        self.user_data = {}

    def __len__(self):
        return self.t

    def get_return(self):
        return self.total_reward


class RLlibCallback:
    """Override any subset of hooks; every hook receives keyword arguments only."""

    def on_algorithm_init(self, *, algorithm, metrics_logger=None, **kwargs):
        pass

    def on_train_result(self, *, algorithm, result: dict, metrics_logger=None, **kwargs):
        pass

    def on_evaluate_start(self, *, algorithm, metrics_logger=None, **kwargs):
        pass

    def on_evaluate_end(self, *, algorithm, evaluation_metrics: dict, metrics_logger=None,
                        **kwargs):
        pass

    def on_checkpoint_loaded(self, *, algorithm, **kwargs):
        pass

    def on_environment_created(self, *, env_runner, env, env_context=None,
                               metrics_logger=None, **kwargs):
        pass

    def on_episode_created(self, *, episode, env_runner=None, env_index=None,
                           metrics_logger=None, **kwargs):
        pass

    def on_episode_start(self, *, episode, env_runner=None, env_index=None,
                         metrics_logger=None, **kwargs):
        pass

    def on_episode_step(self, *, episode, env_runner=None, env_index=None,
                        metrics_logger=None, **kwargs):
        pass

    def on_episode_end(self, *, episode, env_runner=None, env_index=None,
                       metrics_logger=None, **kwargs):
        pass

    def on_sample_end(self, *, env_runner=None, samples=None, metrics_logger=None, **kwargs):
        pass


DefaultCallbacks = RLlibCallback


class _CallbackList(RLlibCallback):
    """Several callback objects behind one (config.callbacks accepts a class, an
    instance, or a list of either)."""

    def __init__(self, cbs):
        self.cbs = cbs

    def __getattribute__(self, name):
        if name.startswith("on_"):
            cbs = object.__getattribute__(self, "cbs")

            def fan(**kw):
                for c in cbs:
                    getattr(c, name)(**kw)

            return fan
        return object.__getattribute__(self, name)


def make_callbacks(spec) -> RLlibCallback:
    if spec is None:
        return RLlibCallback()
    items = spec if isinstance(spec, (list, tuple)) else [spec]
    objs = [c() if isinstance(c, type) else c for c in items]
    return objs[0] if len(objs) == 1 else _CallbackList(objs)
