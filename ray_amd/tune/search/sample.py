"""Search-space primitives (reference: python/ray/tune/search/sample.py, variant_generator.py)."""

from __future__ import annotations

import copy
import itertools
import math
import random


class Domain:
    def sample(self, rng=None, spec=None):
        raise NotImplementedError

    def is_grid(self):
        return False


class Float(Domain):
    def __init__(self, lower, upper, log=False, q=None, normal=None):
        self.lower, self.upper, self.log, self.q, self.normal = lower, upper, log, q, normal

    def sample(self, rng=None, spec=None):
        rng = rng or random
        if self.normal is not None:
            v = rng.gauss(*self.normal)
        elif self.log:
            v = math.exp(rng.uniform(math.log(self.lower), math.log(self.upper)))
        else:
            v = rng.uniform(self.lower, self.upper)
        if self.q:
            v = round(v / self.q) * self.q
        return v


class Integer(Domain):
    def __init__(self, lower, upper, log=False, q=None):
        self.lower, self.upper, self.log, self.q = lower, upper, log, q

    def sample(self, rng=None, spec=None):
        rng = rng or random
        if self.log:
            v = int(math.exp(rng.uniform(math.log(self.lower), math.log(self.upper))))
        else:
            v = rng.randrange(self.lower, self.upper)
        if self.q:
            v = int(round(v / self.q) * self.q)
        return v


class Categorical(Domain):
    def __init__(self, categories):
        self.categories = list(categories)

    def sample(self, rng=None, spec=None):
        return (rng or random).choice(self.categories)


class Function(Domain):
    def __init__(self, fn):
        self.fn = fn

    def sample(self, rng=None, spec=None):
        try:
            return self.fn(spec)
        except TypeError:
            return self.fn()


class Grid(Domain):
    def __init__(self, values):
        self.values = list(values)

    def is_grid(self):
        return True


def uniform(lower, upper):
    return Float(lower, upper)


def quniform(lower, upper, q):
    return Float(lower, upper, q=q)


def loguniform(lower, upper, base=10):
    return Float(lower, upper, log=True)


def qloguniform(lower, upper, q, base=10):
    return Float(lower, upper, log=True, q=q)


def randn(mean=0.0, sd=1.0):
    return Float(None, None, normal=(mean, sd))


def qrandn(mean, sd, q):
    return Float(None, None, normal=(mean, sd), q=q)


def randint(lower, upper):
    return Integer(lower, upper)


def qrandint(lower, upper, q=1):
    return Integer(lower, upper + 1, q=q)


def lograndint(lower, upper, base=10):
    return Integer(lower, upper, log=True)


def qlograndint(lower, upper, q, base=10):
    return Integer(lower, upper, log=True, q=q)


def choice(categories):
    return Categorical(categories)


def sample_from(fn):
    return Function(fn)


def grid_search(values):
    return {"grid_search": list(values)}


def _walk(spec, path=()):
    if isinstance(spec, dict):
        if set(spec.keys()) == {"grid_search"}:
            yield path, Grid(spec["grid_search"])
            return
        for k, v in spec.items():
            yield from _walk(v, path + (k,))
    elif isinstance(spec, Domain):
        yield path, spec


def _set(d, path, v):
    for p in path[:-1]:
        d = d[p]
    d[path[-1]] = v


def generate_variants(spec: dict, num_samples: int = 1, seed=None):
    """Cartesian product of grid_search axes × num_samples random draws."""
    rng = random.Random(seed)
    leaves = list(_walk(spec))
    grids = [(p, d) for p, d in leaves if isinstance(d, Grid)]
    rands = [(p, d) for p, d in leaves if not isinstance(d, Grid)]
    grid_vals = [d.values for _, d in grids] or [[None]]
    for _ in range(num_samples):
        for combo in itertools.product(*grid_vals):
            cfg = copy.deepcopy(spec)
            for (p, _), v in zip(grids, combo):
                _set(cfg, p, v)
            fns = []
            for p, d in rands:
                if isinstance(d, Function):
                    fns.append((p, d))
                else:
                    _set(cfg, p, d.sample(rng))
            for p, d in fns:
                _set(cfg, p, d.sample(rng, _Spec(cfg)))
            yield cfg


class _Spec:
    def __init__(self, cfg):
        self.config = cfg

    def __getattr__(self, k):
        return self.config[k]
