"""Observation filters of the old API stack (reference: python/ray/rllib/utils/filter.py):
``MeanStdFilter`` keeps running mean / variance (Welford), can be applied without updating
(``update=False``), and merges buffered statistics from remote copies
(``apply_changes``). The new stack's connector (connectors/env_to_module.py) and the
learner-side HIP kernel do the same for ray_amd's runners."""

from __future__ import annotations

import numpy as np


class Filter:
    is_concurrent = False

    def __call__(self, x, update: bool = True):
        raise NotImplementedError

    def apply_changes(self, other: "Filter", with_buffer: bool = False, *a, **k):
        pass

    def copy(self) -> "Filter":
        raise NotImplementedError

    def sync(self, other: "Filter") -> None:
        pass

    def reset_buffer(self) -> None:
        pass

    def as_serializable(self) -> "Filter":
        return self.copy()


class NoFilter(Filter):
    is_concurrent = True

    def __call__(self, x, update: bool = True):
        return np.asarray(x) if not isinstance(x, dict) else x

    def copy(self):
        return self


class _RunningStat:
    def __init__(self, shape=()):
        self.n = 0
        self.mean = np.zeros(shape, np.float64)
        self.m2 = np.zeros(shape, np.float64)

    def push_batch(self, x):
        x = np.asarray(x, np.float64)
        if x.ndim == self.mean.ndim:
            x = x[None]
        n = x.shape[0]
        if n == 0:
            return
        bm = x.mean(0)
        bm2 = ((x - bm) ** 2).sum(0)
        tot = self.n + n
        d = bm - self.mean
        self.mean = self.mean + d * n / tot
        self.m2 = self.m2 + bm2 + d ** 2 * self.n * n / tot
        self.n = tot

    def update(self, other: "_RunningStat"):
        if other.n == 0:
            return
        tot = self.n + other.n
        d = other.mean - self.mean
        self.mean = self.mean + d * other.n / tot
        self.m2 = self.m2 + other.m2 + d ** 2 * self.n * other.n / tot
        self.n = tot

    @property
    def std(self):
        var = self.m2 / (self.n - 1) if self.n > 1 else np.square(self.mean)
        return np.sqrt(np.maximum(var, 0.0))

    def copy(self):
        o = _RunningStat(self.mean.shape)
        o.n, o.mean, o.m2 = self.n, self.mean.copy(), self.m2.copy()
        return o


class MeanStdFilter(Filter):
    def __init__(self, shape, demean: bool = True, destd: bool = True, clip: float = 10.0):
        self.shape = tuple(shape) if not isinstance(shape, int) else (shape,)
        self.demean, self.destd, self.clip = demean, destd, clip
        self.running_stats = _RunningStat(self.shape)
        self.buffer = _RunningStat(self.shape)

    def __call__(self, x, update: bool = True):
        x = np.asarray(x, np.float64)
        if update:
            self.running_stats.push_batch(x)
            self.buffer.push_batch(x)
        if self.demean:
            x = x - self.running_stats.mean
        if self.destd:
            x = x / (self.running_stats.std + 1e-8)
        if self.clip:
            x = np.clip(x, -self.clip, self.clip)
        return x

    def apply_changes(self, other: "MeanStdFilter", with_buffer: bool = False, *a, **k):
        self.running_stats.update(other.buffer)
        if with_buffer:
            self.buffer = other.buffer.copy()

    def copy(self):
        o = MeanStdFilter(self.shape, self.demean, self.destd, self.clip)
        o.running_stats = self.running_stats.copy()
        o.buffer = self.buffer.copy()
        return o

    def sync(self, other: "MeanStdFilter") -> None:
        self.running_stats = other.running_stats.copy()
        self.buffer = other.buffer.copy()

    def reset_buffer(self) -> None:
        self.buffer = _RunningStat(self.shape)


class ConcurrentMeanStdFilter(MeanStdFilter):
    is_concurrent = True


def get_filter(filter_config, shape):
    if filter_config == "MeanStdFilter":
        return MeanStdFilter(shape, clip=None)
    if filter_config == "ConcurrentMeanStdFilter":
        return ConcurrentMeanStdFilter(shape, clip=None)
    if filter_config == "NoFilter":
        return NoFilter()
    if callable(filter_config):
        return filter_config(shape)
    raise ValueError(f"Unknown observation_filter: {filter_config}")
