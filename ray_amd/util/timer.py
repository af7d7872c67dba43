"""Windowed duration timer (reference: python/ray/util/timer.py:4 ``_Timer``)."""

from __future__ import annotations

import collections
import time


class _Timer:
    """``with t: ...`` records one duration; ``t.push_units_processed(n)`` the work units.
    Means are over the last `window_size` samples."""

    def __init__(self, window_size: int = 10):
        self._window = window_size
        self._samples = collections.deque(maxlen=window_size)
        self._units = collections.deque(maxlen=window_size)
        self._start = None
        self.count = 0
        self._total = 0.0

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    def start(self):
        self._start = time.perf_counter()

    def stop(self):
        dt = time.perf_counter() - self._start
        self._start = None
        self.push(dt)

    def push(self, dt: float):
        self._samples.append(dt)
        self.count += 1
        self._total += dt

    def push_units_processed(self, n: int):
        self._units.append(n)

    def has_units_processed(self) -> bool:
        return len(self._units) > 0

    @property
    def mean(self) -> float:
        return sum(self._samples) / len(self._samples) if self._samples else 0.0

    @property
    def median(self) -> float:
        s = sorted(self._samples)
        return s[len(s) // 2] if s else 0.0

    @property
    def sum(self) -> float:
        return self._total

    @property
    def mean_units_processed(self) -> float:
        return sum(self._units) / len(self._units) if self._units else 0.0

    @property
    def mean_throughput(self) -> float:
        t = sum(self._samples)
        return sum(self._units) / t if t > 0 else 0.0
