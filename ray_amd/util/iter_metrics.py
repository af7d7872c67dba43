"""``ray.util.iter_metrics`` (reference: python/ray/util/iter_metrics.py): counters and
timers shared along a ``util.iter`` pipeline."""

from __future__ import annotations

import collections
from typing import List

from ray_amd.util.timer import _Timer


class MetricsContext:
    """Metrics of one iterator pipeline: counters, timers, info, and the actors the
    pipeline currently reads from."""

    def __init__(self):
        self.counters = collections.defaultdict(int)
        self.timers = collections.defaultdict(_Timer)
        self.info = {}
        self.current_actor = None

    def save(self):
        return (dict(self.counters), {k: v for k, v in self.timers.items()}, dict(self.info))

    def restore(self, values):
        counters, timers, info = values
        self.counters.clear()
        self.counters.update(counters)
        self.timers.clear()
        self.timers.update(timers)
        self.info = dict(info)


class SharedMetrics:
    """A MetricsContext handed from one pipeline stage to the next (``.get()`` returns it)."""

    def __init__(self, metrics: MetricsContext = None, parents: List["SharedMetrics"] = None):
        self.metrics = metrics or MetricsContext()
        self.parents = parents or []
        self.set(self.metrics)

    def set(self, metrics: MetricsContext):
        self.metrics = metrics
        for p in self.parents:
            p.set(metrics)

    def get(self) -> MetricsContext:
        return self.metrics
