"""Minimal gymnasium-compatible spaces (gymnasium is not installed in this image;
reference RLlib depends on gymnasium.spaces)."""

from __future__ import annotations

import numpy as np


class Space:
    shape = None
    dtype = None

    def __init__(self, seed=None):
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)

    def sample(self):
        raise NotImplementedError

    def contains(self, x) -> bool:
        raise NotImplementedError


class Discrete(Space):
    def __init__(self, n: int, seed=None, start: int = 0):
        super().__init__(seed)
        self.n = int(n)
        self.start = start
        self.shape = ()
        self.dtype = np.int64

    def sample(self):
        return int(self.start + self.np_random.integers(self.n))

    def contains(self, x):
        return int(x) == x and self.start <= x < self.start + self.n

    def __repr__(self):
        return f"Discrete({self.n})"

    def __eq__(self, o):
        return isinstance(o, Discrete) and o.n == self.n


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        super().__init__(seed)
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
        self.shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape)
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape)

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self.np_random.integers(self.low, self.high.astype(np.int64) + 1,
                                           size=self.shape).astype(self.dtype)
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return self.np_random.uniform(lo, hi, size=self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.shape}, {self.dtype})"


class MultiDiscrete(Space):
    def __init__(self, nvec, seed=None):
        super().__init__(seed)
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.int64

    def sample(self):
        return (self.np_random.random(self.nvec.shape) * self.nvec).astype(np.int64)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= 0) and np.all(x < self.nvec))


class Dict(Space):
    def __init__(self, spaces: dict, seed=None):
        super().__init__(seed)
        self.spaces = dict(spaces)

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def contains(self, x):
        return isinstance(x, dict) and all(s.contains(x[k]) for k, s in self.spaces.items())

    def __getitem__(self, k):
        return self.spaces[k]


class Tuple(Space):
    def __init__(self, spaces, seed=None):
        super().__init__(seed)
        self.spaces = tuple(spaces)

    def sample(self):
        return tuple(s.sample() for s in self.spaces)

    def contains(self, x):
        return isinstance(x, tuple) and all(s.contains(v) for s, v in zip(self.spaces, x))
